"""Coset-sharded witness commitment across G GPUs (one process per GPU, RCCL over xGMI).

The reference runs the whole commitment on one host (prover.rs:313-353 with the Worker
pool); this is its multi-GPU split (BASELINE north_star):

  * the trace is column-sharded: rank P holds columns [P*C/G, (P+1)*C/G);
  * each rank inverse-transforms its own columns into the exchange format
    (bj_lde_coeffs_d: monomials in bit-reversed order), straight into its slice of
    the all-columns coefficient buffer;
  * one all-gather (RCCL, in place) gives every rank every column's coefficients
    (8 n C bytes in total) -- the only data-path exchange;
  * rank P evaluates its contiguous range of m = n*D/G leaves of the flat leaf domain
    (coset * n + row, merkle_tree.rs:112-157): whole cosets when G <= D, a folded sub-coset
    when G > D (bj_lde_shard_d);
  * leaves and the subtree over them are hashed locally (contiguous aligned leaf ranges are
    subtrees of the reference's tree, so every node is the reference's node);
  * the cap is all-gathered: cap/G digests per rank when cap >= G; otherwise every rank
    all-gathers the G subtree roots and hashes the top log2(G/cap) levels redundantly.

Outputs stay sharded: each rank keeps its LDE slice, its leaves and subtree nodes, and
the full cap.  The compute steps are an `ops` object: `HipShardOps` (the C ABI on the
GPU) is the product path and the default; the CPU multi-process tests inject a CPU
implementation to check the orchestration with `gloo`.
"""
import torch

from ._lib import call
from .field import stream_of


def _log2(n):
    if n <= 0 or n & (n - 1):
        raise ValueError("size must be a power of two, got %d" % n)
    return n.bit_length() - 1


class HipShardOps:
    """The product compute steps, through libboojum_mi355x.so on the current stream."""

    def coeffs(self, trace, out, log_n):
        call("bj_lde_coeffs_d", trace.data_ptr(), trace.shape[0], trace.stride(0), log_n, out.data_ptr(),
             out.stride(0), stream_of(out))

    def lde_shard(self, coeffs, log_n, log_lde, log_shards, shard, work, lde):
        call("bj_lde_shard_d", coeffs.data_ptr(), coeffs.shape[0], coeffs.stride(0), log_n, log_lde, log_shards,
             shard, None if work is None else work.data_ptr(), lde.data_ptr(), stream_of(lde))

    def leaves(self, lde, out):
        c, m = lde.shape
        call("bj_merkle_leaves_d", lde.data_ptr(), c, lde.stride(0), m, out.data_ptr(), stream_of(out))

    def nodes(self, leaves, cap_size, out):
        call("bj_merkle_nodes_d", leaves.data_ptr(), leaves.shape[0], cap_size, out.data_ptr(), stream_of(out))

    def synthetic(self, out, log_n, first_col):
        call("bj_fill_synthetic_d", out.data_ptr(), out.shape[0], out.stride(0), log_n, 42, first_col,
             stream_of(out))


def _all_gather(out, inp, group=None):
    """out (G*k, ...) <- concat over ranks of inp (k, ...).  RCCL (backend "nccl") runs in
    place on device memory; gloo (the CPU tests) stages device tensors through the host."""
    import torch.distributed as dist
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, inp, group=group)
        return
    world = dist.get_world_size(group)
    src = inp.detach().cpu().contiguous()
    parts = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(parts, src, group=group)
    out.copy_(torch.cat(parts, 0).to(out.device))


class ShardedWorkspace:
    """Per-rank HBM buffers of a G-way sharded commit of C x 2^log_n at LDE 2^log_lde.

    coeffs (C, n)             all columns' coefficients (this rank's slice written locally)
    work   (C, m) | None      fold scratch (G > D only)
    lde    (C, m)             this rank's leaf range of every column's LDE, m = n*D/G
    leaves (m, 4), nodes (m - cap_local, 4), cap (cap, 4)
    """

    def __init__(self, n_cols, log_n, log_lde, cap_size, rank, world, device="cuda", group=None, ops=None):
        log_g = _log2(world)
        _log2(cap_size)
        if n_cols % world:
            raise ValueError("n_cols (%d) must be a multiple of the number of shards (%d)" % (n_cols, world))
        if log_g > log_n + log_lde:
            raise ValueError("more shards than leaves")
        if log_lde == 0:
            raise ValueError("lde degree must be > 1 (utils.rs:283)")
        if cap_size >= (1 << (log_n + log_lde)):
            raise ValueError("tree size must exceed cap size")
        self.n_cols, self.log_n, self.log_lde, self.cap_size = n_cols, log_n, log_lde, cap_size
        self.rank, self.world, self.log_g, self.group = rank, world, log_g, group
        self.ops = ops if ops is not None else HipShardOps()
        n = 1 << log_n
        self.m = m = (n << log_lde) >> log_g
        self.cols_per_rank = n_cols // world
        self.cap_local = max(1, cap_size // world)
        if m <= self.cap_local:
            raise ValueError("each shard needs more leaves than its cap slice")
        kw = dict(dtype=torch.int64, device=device)
        self.coeffs = torch.empty((n_cols, n), **kw)
        self.work = torch.empty((n_cols, m), **kw) if log_g > log_lde else None
        self.lde = torch.empty((n_cols, m), **kw)
        self.leaves = torch.empty((m, 4), **kw)
        self.nodes = torch.empty((m - self.cap_local, 4), **kw)
        self.cap = torch.empty((cap_size, 4), **kw)
        if cap_size < world:
            self.roots = torch.empty((world, 4), **kw)
            self.top_nodes = torch.empty((world - cap_size, 4), **kw)
        if hasattr(self.ops, "prepare"):
            self.ops.prepare(log_n)
        elif self.coeffs.is_cuda:
            call("bj_prepare", log_n)

    @property
    def my_columns(self):
        c0 = self.rank * self.cols_per_rank
        return c0, c0 + self.cols_per_rank

    @property
    def leaf_range(self):
        return self.rank * self.m, (self.rank + 1) * self.m

    def synthetic_trace_shard(self):
        """This rank's columns of the synthetic trace, generated in place."""
        t = torch.empty((self.cols_per_rank, 1 << self.log_n), dtype=torch.int64, device=self.coeffs.device)
        self.ops.synthetic(t, self.log_n, self.my_columns[0])
        return t


def sharded_witness_commit(trace_shard, ws, marks=None):
    """Commit this rank's column shard (C/G, n) into `ws`; collective over ws.group.

    `marks`, if given, is called with a phase name after each phase is enqueued
    ("ifft", "exchange", "lde", "leaves", "nodes") -- the bench records events there."""
    ops = ws.ops
    mark = marks or (lambda name: None)
    c0, c1 = ws.my_columns
    if tuple(trace_shard.shape) != (ws.cols_per_rank, 1 << ws.log_n):
        raise ValueError("trace shard must be (%d, %d)" % (ws.cols_per_rank, 1 << ws.log_n))
    mine = ws.coeffs[c0:c1]
    ops.coeffs(trace_shard, mine, ws.log_n)
    mark("ifft")
    if ws.world > 1:
        _all_gather(ws.coeffs, mine, ws.group)
    mark("exchange")
    ops.lde_shard(ws.coeffs, ws.log_n, ws.log_lde, ws.log_g, ws.rank, ws.work, ws.lde)
    mark("lde")
    ops.leaves(ws.lde, ws.leaves)
    mark("leaves")
    ops.nodes(ws.leaves, ws.cap_local, ws.nodes)
    local_cap = ws.nodes[-ws.cap_local:]
    if ws.cap_size >= ws.world:
        if ws.world > 1:
            _all_gather(ws.cap, local_cap, ws.group)
        else:
            ws.cap.copy_(local_cap)
    else:
        _all_gather(ws.roots, local_cap, ws.group)
        ops.nodes(ws.roots, ws.cap_size, ws.top_nodes)
        ws.cap.copy_(ws.top_nodes[-ws.cap_size:])
    mark("nodes")
    return ws
