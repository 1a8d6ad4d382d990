"""FRI folding of the DEEP codeword (cs/implementations/fri/mod.rs:179-300) on the GPU.

The codeword is a GoldilocksExt2 vector held as two base columns c0, c1 over the full LDE
domain, bit-reversed (cosets one after another). One fold by 2 (`fold`, bj_fri_fold_d)
is fold_multiple (fri/mod.rs:362-474). `interpolate` chains folds the way
interpolate_independent_cosets / interpolate_flattened_cosets (:476-682) do:
* the root table is the INVERSED bit-reversed twiddles of the full domain;
* it is indexed by the flat pair index at every step;
* the coset inverse starts at 7^-1 (fri/mod.rs:194) and is squared after each fold.

The oracles over the folded vectors are MerkleTreeWithCap.construct_by_chunking(_from_flat_sources)
(merkle.py). The transcript that draws the challenges is outside this path; challenges are
inputs. Scalar setup (challenge powers, the coset inverse) is host arithmetic on single
field elements, as in the reference's own driver loop.
"""
import torch

from ._lib import call
from .field import GENERATOR, P, stream_of

EXT2_NON_RESIDUE = 7   # GoldilocksExt2::NON_RESIDUE (field/goldilocks/extension.rs:14-16)


def _log2(n):
    if n <= 0 or n & (n - 1):
        raise ValueError("size must be a power of two, got %d" % n)
    return n.bit_length() - 1


def ext2_square(a):
    """(a0 + a1 u)^2 with u^2 = 7 (field/traits/field.rs:427-440), on host ints."""
    a0, a1 = a
    return ((a0 * a0 + EXT2_NON_RESIDUE * a1 * a1) % P, (2 * a0 * a1) % P)


def challenge_powers(challenge, reduction_degree_log_2):
    """[alpha, alpha^2, alpha^4, ...] as fri/mod.rs:206-226 builds them for one reduction step."""
    out = [(challenge[0] % P, challenge[1] % P)]
    for _ in range(1, reduction_degree_log_2):
        out.append(ext2_square(out[-1]))
    return out


def precompute_roots(full_size, device="cuda"):
    """precompute_twiddles_for_fft::<INVERSED = true>(full_size) (fri/mod.rs:191-192)."""
    log_n = _log2(full_size)
    out = torch.empty((full_size // 2,), dtype=torch.int64, device=device)
    call("bj_precompute_twiddles_d", log_n, 1, out.data_ptr(), stream_of(out))
    return out


def fold(c0, c1, roots, coset_inverse, challenge):
    """One fold by 2: (N,) device columns -> (N/2,) each."""
    n = c0.shape[-1]
    if c1.shape[-1] != n or roots.shape[-1] < n // 2:
        raise ValueError("c0, c1 and roots sizes do not match")
    d0 = torch.empty((n // 2,), dtype=torch.int64, device=c0.device)
    d1 = torch.empty_like(d0)
    call("bj_fri_fold_d", c0.data_ptr(), c1.data_ptr(), n, roots.data_ptr(), coset_inverse % P, challenge[0] % P,
         challenge[1] % P, d0.data_ptr(), d1.data_ptr(), stream_of(c0))
    return d0, d1


def interpolate(c0, c1, challenges, roots, coset_inverse=None):
    """Fold len(challenges) times (interpolate_independent_cosets + interpolate_flattened_cosets).
    c0, c1: (N,) flat bit-reversed codeword columns (cosets in order). Returns
    (c0', c1', coset_inverse after the folds)."""
    ci = pow(GENERATOR, P - 2, P) if coset_inverse is None else coset_inverse % P
    for ch in challenges:
        c0, c1 = fold(c0.reshape(-1), c1.reshape(-1), roots, ci, ch)
        ci = ci * ci % P
    return c0, c1, ci
