"""Reference-named FFT entry points over the HIP library.

Mirrors the reference's `src/fft` surface (fft/mod.rs:308-491, 625-657) and the
PrimeFieldLikeVectorized seam (field/traits/field_like.rs:111-162):

* device form: torch CUDA tensors of dtype int64 holding u64 bit patterns, shape (n,)
  or (C, n) (a batch of columns, one call instead of the reference's per-column rayon
  tasks, cs/implementations/utils.rs:295-304,363-379);
* host form (`*_host`): numpy uint64 arrays, in place, synchronous -- the exact
  per-call contract of the Rust seam.

Errors: preconditions the reference asserts (power-of-two sizes, fft/mod.rs:399-402)
raise BoojumError / ValueError.  There is no CPU fallback.
"""
import ctypes

import numpy as np

from ._lib import call
from .field import as_u64_host, col_view, stream_of

_u64p = ctypes.POINTER(ctypes.c_uint64)


def _log2(n):
    if n <= 0 or n & (n - 1):
        raise ValueError("size must be a power of two, got %d" % n)
    return n.bit_length() - 1


# ---------------------------------------------------------------- device forms

def precompute_twiddles_for_fft(fft_size, inverse=False, device=None):
    """precompute_twiddles_for_fft::<INVERSED> (utils.rs:88-125): omega^i (omega^-i),
    i < n/2, bit-reversed.  Returns an int64 CUDA tensor of n/2 u64."""
    import torch
    log_n = _log2(fft_size)
    if log_n == 0:
        raise ValueError("twiddles need fft_size >= 2")
    out = torch.empty(fft_size // 2, dtype=torch.int64, device=device or "cuda")
    call("bj_precompute_twiddles_d", log_n, 1 if inverse else 0, out.data_ptr(), stream_of(out))
    return out


def fft_natural_to_bitreversed(cols, coset=1, twiddles=None):
    """fft/mod.rs:398-411, in place on a (n,) or (C, n) int64 CUDA tensor."""
    v, c, n, stride = col_view(cols)
    call("bj_fft_natural_to_bitreversed_d", v.data_ptr(), c, stride, _log2(n), int(coset),
         twiddles.data_ptr() if twiddles is not None else None, stream_of(v))
    return cols


def ifft_natural_to_natural(cols, coset=1, twiddles=None):
    """fft/mod.rs:464-491, in place."""
    v, c, n, stride = col_view(cols)
    call("bj_ifft_natural_to_natural_d", v.data_ptr(), c, stride, _log2(n), int(coset),
         twiddles.data_ptr() if twiddles is not None else None, stream_of(v))
    return cols


def distribute_powers(cols, element):
    """fft/mod.rs:308-317, in place: col[j] *= element^j."""
    v, c, n, stride = col_view(cols)
    call("bj_distribute_powers_d", v.data_ptr(), c, stride, _log2(n), int(element), stream_of(v))
    return cols


def precompute_twiddles_for_fft_natural(fft_size, inverse=False, device=None):
    """precompute_twiddles_for_fft_natural::<INVERSED> (utils.rs:127-155, fft/mod.rs:640-657):
    omega^i (omega^-i), i < n/2, natural order.  int64 CUDA tensor of n/2 u64."""
    import torch
    log_n = _log2(fft_size)
    if log_n == 0:
        raise ValueError("twiddles need fft_size >= 2")
    out = torch.empty(fft_size // 2, dtype=torch.int64, device=device or "cuda")
    call("bj_precompute_twiddles_natural_d", log_n, 1 if inverse else 0, out.data_ptr(), stream_of(out))
    return out


def bitreverse_enumeration_inplace(cols):
    """fft/mod.rs:41-155: bit-reversal permutation of each column, in place."""
    v, c, n, stride = col_view(cols)
    call("bj_bitreverse_enumeration_d", v.data_ptr(), c, stride, _log2(n), stream_of(v))
    return cols


# The reference's cache-friendly and MixedGL (SIMD-packed) variants compute the same transform
# with another loop order or lane packing (fft/mod.rs:413-462, 493-623); on the GPU they are the
# same batched kernels.
fft_natural_to_bitreversed_cache_friendly = fft_natural_to_bitreversed
fft_natural_to_bitreversed_mixedgl = fft_natural_to_bitreversed
fft_natural_to_bitreversed_mixedgl_interleaving = fft_natural_to_bitreversed
ifft_natural_to_natural_cache_friendly = ifft_natural_to_natural
ifft_natural_to_natural_mixedgl = ifft_natural_to_natural
ifft_natural_to_natural_mixedgl_interleaving = ifft_natural_to_natural
precompute_twiddles_for_fft_wrapper = precompute_twiddles_for_fft
precompute_twiddles_for_fft_natural_wrapper = precompute_twiddles_for_fft_natural


# ------------------------------------------------------------------ host forms

def _hp(a):
    return a.ctypes.data_as(_u64p)


def precompute_twiddles_for_fft_host(fft_size, inverse=False):
    log_n = _log2(fft_size)
    out = np.zeros(fft_size // 2, dtype=np.uint64)
    call("bj_precompute_twiddles_h", log_n, 1 if inverse else 0, _hp(out))
    return out


def fft_natural_to_bitreversed_host(col, coset=1):
    a = as_u64_host(col)
    _log2(a.size)
    call("bj_fft_natural_to_bitreversed_h", _hp(a), a.size, int(coset))
    return a


def ifft_natural_to_natural_host(col, coset=1):
    a = as_u64_host(col)
    _log2(a.size)
    call("bj_ifft_natural_to_natural_h", _hp(a), a.size, int(coset))
    return a


def distribute_powers_host(col, element):
    a = as_u64_host(col)
    _log2(a.size)
    call("bj_distribute_powers_h", _hp(a), a.size, int(element))
    return a
