"""The witness-commitment hot path as one batched call.

`witness_commit` = prover.rs:313-353: LDE of every column at D = used_lde_degree
(transform_raw_storages_to_lde), MerkleTreeWithCap::construct over the rows of the first
k = fri_lde_factor cosets (subset_for_degree, prover.rs:325-347; k = D unless given), get_cap.
`CommitWorkspace` preallocates every HBM buffer once so repeated commits (the bench loop, a
prover running many circuits) never allocate.
"""
import torch

from ._lib import call
from .field import col_view, stream_of


def _log2(n):
    if n <= 0 or n & (n - 1):
        raise ValueError("size must be a power of two, got %d" % n)
    return n.bit_length() - 1


class CommitWorkspace:
    """HBM buffers for a commit of n_cols x 2^log_n at LDE 2^log_lde, tree over the first
    k = 2^log_commit_cosets cosets (default k = D), cap cap_size.

    Sizes (bytes): scratch 8*C*n, lde 8*C*n*D, leaves 32*n*k, nodes 32*(n*k - cap)."""

    def __init__(self, n_cols, log_n, log_lde, cap_size, device="cuda", log_commit_cosets=None):
        log_k = log_lde if log_commit_cosets is None else log_commit_cosets
        if not 0 <= log_k <= log_lde:
            raise ValueError("committed cosets must not exceed the LDE degree")
        n, d = 1 << log_n, 1 << log_lde
        nl = n << log_k
        _log2(cap_size)
        if nl <= cap_size:
            raise ValueError("tree size must exceed cap size")
        self.n_cols, self.log_n, self.log_lde, self.cap_size = n_cols, log_n, log_lde, cap_size
        self.log_k = log_k
        self.scratch = torch.empty((n_cols, n), dtype=torch.int64, device=device)
        self.lde = torch.empty((n_cols, d, n), dtype=torch.int64, device=device)
        self.leaves = torch.empty((nl, 4), dtype=torch.int64, device=device)
        self.nodes = torch.empty((nl - cap_size, 4), dtype=torch.int64, device=device)
        call("bj_prepare", log_n)

    @property
    def cap(self):
        return self.nodes[-self.cap_size:]

    def tree(self):
        from .merkle import MerkleTreeWithCap
        return MerkleTreeWithCap(self.cap_size, self.leaves, self.nodes, getattr(self, "hasher", "poseidon2"))


def witness_commit(trace, lde_degree, cap_size, workspace=None, hasher="poseidon2", fri_lde_factor=None):
    """Commit a (C, n) int64 CUDA trace tensor: LDE at lde_degree (D), tree over the first
    fri_lde_factor (k, default D) cosets.  Returns the workspace holding lde (C, D, n), leaves
    (k n, 4), nodes and cap (all on device, canonical).  Asynchronous on the current stream.
    hasher: "poseidon2" (GoldilocksPoseidon2Sponge, the recursive-mode tree), "blake2s"
    (Blake2s256, the non-recursive one) or "keccak256"."""
    v, c, n, stride = col_view(trace)
    log_n, log_d = _log2(n), _log2(lde_degree)
    log_k = log_d if fri_lde_factor is None else _log2(fri_lde_factor)
    ws = workspace or CommitWorkspace(c, log_n, log_d, cap_size, device=v.device, log_commit_cosets=log_k)
    if (ws.n_cols, ws.log_n, ws.log_lde, ws.log_k, ws.cap_size) != (c, log_n, log_d, log_k, cap_size):
        raise ValueError("workspace shape does not match the trace")
    st = stream_of(v)
    if hasher == "poseidon2":
        call("bj_lde_commit_d", v.data_ptr(), c, stride, log_n, log_d, log_k, cap_size, ws.scratch.data_ptr(),
             ws.lde.data_ptr(), ws.leaves.data_ptr(), ws.nodes.data_ptr(), None, st)
    else:
        from .merkle import HASHERS
        if hasher not in HASHERS:
            raise ValueError("unknown tree hasher %r" % (hasher,))
        _, f_leaves, _, f_nodes = HASHERS[hasher]
        nd, nl = n << log_d, n << log_k
        call("bj_lde_ex_d", v.data_ptr(), c, stride, log_n, log_d, ws.scratch.data_ptr(), ws.lde.data_ptr(), 0, st)
        call(f_leaves, ws.lde.data_ptr(), c, nd, nl, ws.leaves.data_ptr(), st)
        call(f_nodes, ws.leaves.data_ptr(), nl, cap_size, ws.nodes.data_ptr(), st)
    ws.hasher = hasher
    return ws


class CommitGraph:
    """The whole commit of a fixed trace buffer, captured once as a HIP graph and replayed.

    A prover that commits many traces of one shape (or the bench) refills `trace` in place and
    calls replay(): one graph launch instead of the commit's ~10-30 kernel launches, which is
    what bounds the small shapes (C1, C5). The first commit runs eagerly, outside the capture,
    so every twiddle / power table the kernels read is created (and cached) before capturing;
    the captured calls then only launch kernels on the capture stream."""

    def __init__(self, trace, lde_degree, cap_size, hasher="poseidon2", workspace=None):
        self.trace = trace
        self.args = (lde_degree, cap_size)
        self.hasher = hasher
        self.ws = witness_commit(trace, lde_degree, cap_size, workspace, hasher)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            witness_commit(trace, lde_degree, cap_size, self.ws, hasher)

    def replay(self):
        """Commit the current contents of `trace` (asynchronous on the current stream)."""
        self.graph.replay()
        return self.ws


def synthetic_trace(n_cols, log_n, seed=42, first_col=0, device="cuda", out=None):
    """Device-generated synthetic trace: splitmix64(seed + c*n + r) mod p."""
    n = 1 << log_n
    t = out if out is not None else torch.empty((n_cols, n), dtype=torch.int64, device=device)
    call("bj_fill_synthetic_d", t.data_ptr(), n_cols, n, log_n, seed, first_col, stream_of(t))
    return t


# ------------------------------------------------------------------ other oracles
# The prover's other commitments go through the same kernels; only the column sets and the
# LDE degree vs committed cosets differ.  The reference computes every LDE at
# used_lde_degree = max(fri_lde_factor, quotient_degree) (prover.rs:313) and commits only the
# first fri_lde_factor cosets of each column (subset_for_degree, lde.rs:298-308).


class OracleCommitment:
    """An LDE (C, D, n) on device and the MerkleTreeWithCap over its first k cosets."""

    def __init__(self, lde, tree):
        self.lde = lde
        self.tree = tree

    def get_cap(self):
        return self.tree.get_cap()


def commit_trace_columns(trace, lde_degree, fri_lde_factor, cap_size, hasher="poseidon2"):
    """Base-field columns (C, n) in Lagrange (trace) form: iFFT, coset LDE at lde_degree, tree
    over the first fri_lde_factor cosets, as one batched commit (bj_lde_commit_d).  The witness
    oracle (prover.rs:316-347) and the setup oracle (setup.rs:1146-1204, setup_storage.rs:18-70)
    are this call."""
    from .merkle import MerkleTreeWithCap
    if fri_lde_factor > lde_degree:
        raise ValueError("fri_lde_factor exceeds the LDE degree")
    t = torch.as_tensor(trace)
    if not t.is_cuda:
        t = t.to("cuda")
    ws = witness_commit(t, lde_degree, cap_size, hasher=hasher, fri_lde_factor=fri_lde_factor)
    return OracleCommitment(ws.lde, MerkleTreeWithCap(cap_size, ws.leaves, ws.nodes, hasher))


def second_stage_commit(z_poly, intermediate_polys, lookup_witness_encoding_polys,
                        lookup_multiplicities_encoding_polys, lde_degree, fri_lde_factor, cap_size,
                        hasher="poseidon2"):
    """SecondStageProductsStorage::from_base_trace_ext + the stage-2 tree (prover.rs:505-554).
    Every argument is a GoldilocksExt2 polynomial as a (c0, c1) pair of (n,) base columns in
    Lagrange form (or a list of such pairs); the leaf order is z, intermediates, lookup witness
    encodings, multiplicity encodings, each as c0 then c1 (prover.rs:520-547)."""
    cols = [z_poly[0], z_poly[1]]
    for group in (intermediate_polys, lookup_witness_encoding_polys, lookup_multiplicities_encoding_polys):
        for c0, c1 in group:
            cols += [c0, c1]
    trace = torch.stack([torch.as_tensor(c) for c in cols])
    return commit_trace_columns(trace, lde_degree, fri_lde_factor, cap_size, hasher=hasher)


def quotient_commit(monomials, fri_lde_factor, cap_size, hasher="poseidon2"):
    """Quotient chunks already in monomial form (prover.rs:1454-1495): transform_monomials_to_lde
    at fri_lde_factor, then the tree over all its cosets."""
    from .lde import transform_monomials_to_lde
    from .merkle import MerkleTreeWithCap
    lde = transform_monomials_to_lde(monomials, fri_lde_factor)
    return OracleCommitment(lde, MerkleTreeWithCap.construct(lde, cap_size, hasher=hasher))
