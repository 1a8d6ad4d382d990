"""Goldilocks constants and the tensor plumbing shared by the host-side API.

Device data is held in torch CUDA tensors of dtype int64 whose bits are the u64 field
representatives (torch is used for HBM allocation and streams only; every computation
is a HIP kernel behind the C ABI).
"""
import numpy as np

P = 0xFFFFFFFF00000001          # field/goldilocks/mod.rs:111
GENERATOR = 7                   # MULTIPLICATIVE_GROUP_GENERATOR, mod.rs:107
ROOT_OF_UNITY_2_32 = 0x185629dcda58878c  # RADIX_2_SUBGROUP_GENERATOR, mod.rs:108
TWO_ADICITY = 32


def as_u64_host(a):
    """numpy uint64 C-contiguous array (the same object if it already is one, so the
    *_host seam functions really are in place for such inputs)."""
    if isinstance(a, np.ndarray) and a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"]:
        return a
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint64))


def stream_of(t):
    import torch
    return torch.cuda.current_stream(t.device).cuda_stream


def col_view(t):
    """(tensor, n_cols, n, col_stride) for an int64 CUDA tensor of shape (n,) or (C, n)
    whose rows are unit-stride."""
    import torch
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError("expected a CUDA tensor")
    if t.dtype not in (torch.int64, torch.uint64):
        raise TypeError("expected int64/uint64 storage of u64 field elements")
    if t.dim() == 1:
        t2 = t.unsqueeze(0)
    elif t.dim() == 2:
        t2 = t
    else:
        raise ValueError("expected shape (n,) or (C, n)")
    if t2.stride(1) != 1:
        raise ValueError("columns must be contiguous")
    c, n = t2.shape
    stride = t2.stride(0) if c > 1 else n
    return t2, c, n, stride


def to_device(a, device="cuda"):
    """numpy uint64 -> int64 CUDA tensor with the same bits."""
    import torch
    a = np.ascontiguousarray(np.asarray(a, dtype=np.uint64))
    return torch.from_numpy(a.view(np.int64)).to(device)


def to_host(t):
    """int64 CUDA tensor -> numpy uint64 (same bits)."""
    return t.detach().cpu().contiguous().numpy().view(np.uint64)
