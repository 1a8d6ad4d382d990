"""LDE storage drivers, mirroring cs/implementations/utils.rs:160-403 and the
"worker-driven LDE storage" of witness_storage.rs / setup_storage.rs.

Layout in HBM: trace (C, n); monomials (C, n); LDE (C, D, n) -- column-major, each
column holding its D cosets back to back, each coset in bit-reversed row order
(polynomial/lde.rs:156-346).  The flat leaf index of the Merkle tree over the LDE is
L = coset * n + row, so column c's leaf-domain values are the contiguous row
lde[c].reshape(-1).
"""
import torch

from ._lib import call
from .field import col_view, stream_of


def lde_coset(log_n, log_d, i):
    """7 * w_{nD}^{bitrev_{log D}(i)} (utils.rs:334-347, 370-373)."""
    from .field import GENERATOR, P, ROOT_OF_UNITY_2_32
    g = ROOT_OF_UNITY_2_32
    for _ in range(log_n + log_d, 32):
        g = g * g % P
    r = int(format(i, "0%db" % log_d)[::-1], 2) if log_d else 0
    return pow(g, r, P) * GENERATOR % P


def _log2(n):
    if n <= 0 or n & (n - 1):
        raise ValueError("size must be a power of two, got %d" % n)
    return n.bit_length() - 1


def transform_raw_storages_to_lde(trace, lde_degree, scratch=None, out=None):
    """utils.rs:270-309 + transform_monomials_to_lde :311-403 for a (C, n) int64 CUDA
    tensor.  Returns lde (C, D, n) (the reference returns only the LDE storages; the
    monomials are consumed).  `scratch` (C, n) / `out` may be preallocated buffers
    (reused across calls by a batched prover)."""
    v, c, n, stride = col_view(trace)
    log_n, log_d = _log2(n), _log2(lde_degree)
    if log_d == 0:
        raise ValueError("lde_degree must be > 1 (utils.rs:283)")
    if scratch is None:
        scratch = torch.empty((c, n), dtype=torch.int64, device=v.device)
    if out is None:
        out = torch.empty((c, lde_degree, n), dtype=torch.int64, device=v.device)
    # the monomials are not kept (flags 0): scratch is workspace only, as the reference drops them
    call("bj_lde_ex_d", v.data_ptr(), c, stride, log_n, log_d, scratch.data_ptr(), out.data_ptr(), 0, stream_of(v))
    return out


def transform_monomials_to_lde(monomials, lde_degree, out=None):
    """utils.rs:311-403 (also the quotient commit, prover.rs:1471-1482)."""
    v, c, n, stride = col_view(monomials)
    log_n, log_d = _log2(n), _log2(lde_degree)
    if log_d == 0:
        raise ValueError("lde_degree must be > 1 (utils.rs:283)")
    if out is None:
        out = torch.empty((c, lde_degree, n), dtype=torch.int64, device=v.device)
    call("bj_monomials_to_lde_d", v.data_ptr(), c, stride, log_n, log_d, out.data_ptr(), stream_of(v))
    return out


class ArcGenericLdeStorage:
    """Per-column LDE storage view (polynomial/lde.rs:156-341): `storage[i]` is coset i
    of this column (bit-reversed rows).  Backed by one (D, n) slice of the batch tensor."""

    def __init__(self, cosets):
        self.cosets = cosets  # (D, n) tensor view

    @property
    def storage(self):
        return [self.cosets[i] for i in range(self.cosets.shape[0])]

    def outer_len(self):
        return self.cosets.shape[0]

    def inner_len(self):
        return self.cosets.shape[1]

    def subset_for_degree(self, degree):
        """First `degree` cosets (lde.rs:298-308)."""
        return ArcGenericLdeStorage(self.cosets[:degree])


class WitnessStorage:
    """WitnessStorage::from_base_trace (witness_storage.rs:18-116): the LDE of the
    variables/witness/multiplicity columns at `used_lde_degree`."""

    def __init__(self, lde):
        self.lde = lde

    @classmethod
    def from_base_trace(cls, trace, lde_degree):
        return cls(transform_raw_storages_to_lde(trace, lde_degree))

    def columns(self):
        return [ArcGenericLdeStorage(self.lde[c]) for c in range(self.lde.shape[0])]
