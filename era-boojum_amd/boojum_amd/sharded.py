"""Coset-sharded witness commitment across G GPUs (one process per GPU, RCCL over xGMI).

The reference runs the whole commitment on one host (prover.rs:313-353 with the Worker
pool). This is its multi-GPU split (BASELINE north_star):

  * the trace is column-sharded: every rank holds C/G of the columns;
  * each rank inverse-transforms its own columns into the exchange format
    (bj_lde_coeffs_d: monomials in bit-reversed order), straight into its slice of the
    all-columns coefficient buffer;
  * G <= D: all-gathers (RCCL, in place) give every rank every column's coefficients
    (8 n C bytes in total); rank P evaluates its whole cosets (bj_lde_shard_d);
  * G > D: rank P's m = n*D/G leaves are a sub-coset, whose evaluation only needs every column
    folded mod Y^m - s_P^m (m values instead of n). The sender folds its own columns for every
    rank at once (bj_lde_fold_shards_d) and one all-to-all per chunk delivers them
    (8 m C bytes in total, G/D times less than the all-gather); rank P transforms what it
    received (bj_lde_shard_folded_d). These collectives are the only data-path exchange;
  * rank P's range of the flat leaf domain (coset * n + row, merkle_tree.rs:112-157) is
    [P m, (P+1) m);
  * leaves and the subtree over them are hashed locally. Contiguous aligned leaf ranges are
    subtrees of the reference's tree, so every node is the reference's node;
  * the cap is all-gathered: cap/G digests per rank when cap >= G. Otherwise every rank
    all-gathers the G subtree roots and hashes the top log2(G/cap) levels redundantly.

Column pipeline. The leaf sponge absorbs columns in order, 8 per permutation, and between
8-column groups its only carried state is the 4 capacity words (bj_merkle_leaves_partial_d).
So the columns are dealt out chunk by chunk: chunk k is G c_k consecutive columns (a multiple
of 8), of which rank P holds the P-th run of c_k; c = u, u, 2u, 4u, ... capped at
MAX_CHUNK_COLS, u = 8 / gcd(8, G) (so the first chunk is only 8 columns wide). Each chunk's
exchange is issued on RCCL's stream as soon as this rank's part of it is inverse-transformed
(and folded). Chunk k's coset transform and sponge absorption then run on the compute stream
as soon as chunk k has arrived, while later chunks are still on the wire. Rank P's run of
chunk k is global columns [G S_k + P c_k, G S_k + (P+1) c_k), local [S_k, S_k + c_k),
S_k = c_0 + ... + c_{k-1}. If C/G is not a multiple of u, rank P holds the contiguous
columns [P*C/G, (P+1)*C/G) and one exchange runs before the transforms.

Outputs stay sharded: each rank keeps its LDE slice, its leaves and subtree nodes, and
the full cap. The compute steps are an `ops` object: `HipShardOps` (the C ABI on the
GPU) is the product path and the default; the CPU multi-process tests inject a CPU
implementation to check the orchestration with `gloo`.
"""
import math

import torch

from ._lib import call
from .field import stream_of

MAX_CHUNK_COLS = 32   # largest pipelined chunk, in columns per rank


def _chunk_unit(world):
    """Fewest columns per rank that make a chunk a whole number of 8-column sponge groups."""
    return 8 // math.gcd(8, world)


def _chunk_schedule(cols_per_rank, unit, max_cols=MAX_CHUNK_COLS):
    """Columns per rank in each pipelined chunk: u, u, 2u, 4u, ... capped at max_cols (rounded
    to a multiple of u).  The first chunks are small so little of the exchange is exposed before
    the pipeline fills; later ones are larger so the per-chunk launch and tail costs stay small."""
    max_cols = max(unit, max_cols // unit * unit)
    sched, done, b = [], 0, unit
    while done < cols_per_rank:
        take = min(b, cols_per_rank - done)
        sched.append(take)
        done += take
        if len(sched) >= 2:
            b = min(2 * b, max_cols)
    return sched


def _log2(n):
    if n <= 0 or n & (n - 1):
        raise ValueError("size must be a power of two, got %d" % n)
    return n.bit_length() - 1


# tree hashers whose leaf message can be continued over column ranges (the column pipeline)
PARTIAL_HASHERS = ("poseidon2", "blake2s")


class HipShardOps:
    """The product compute steps, through libboojum_mi355x.so on the current stream.
    hasher: the MerkleTreeWithCap tree hasher (boojum_amd.merkle.HASHERS)."""

    def __init__(self, hasher="poseidon2"):
        from .merkle import HASHERS
        if hasher not in HASHERS:
            raise ValueError("unknown tree hasher %r" % (hasher,))
        self.hasher = hasher
        self._leaves_fn, self._nodes_fn = HASHERS[hasher][1], HASHERS[hasher][3]

    def coeffs(self, trace, out, log_n):
        call("bj_lde_coeffs_d", trace.data_ptr(), trace.shape[0], trace.stride(0), log_n, out.data_ptr(),
             out.stride(0), stream_of(out))

    def fold_shards(self, coeffs, log_n, log_lde, log_shards, out):
        g, c, m = out.shape
        call("bj_lde_fold_shards_d", coeffs.data_ptr(), coeffs.shape[0], coeffs.stride(0), log_n, log_lde, log_shards,
             out.data_ptr(), out.stride(0), stream_of(out))

    def lde_shard_folded(self, folded, log_n, log_lde, log_shards, shard, lde):
        call("bj_lde_shard_folded_d", folded.data_ptr(), folded.shape[0], folded.stride(0), log_n, log_lde,
             log_shards, shard, lde.data_ptr(), stream_of(lde))

    def lde_shard(self, coeffs, log_n, log_lde, log_shards, shard, work, lde):
        call("bj_lde_shard_d", coeffs.data_ptr(), coeffs.shape[0], coeffs.stride(0), log_n, log_lde, log_shards,
             shard, None if work is None else work.data_ptr(), lde.data_ptr(), stream_of(lde))

    def leaves(self, lde, out, cap_in=None, final=True, cols_before=0):
        """Leaf messages over the column range lde (C_k, m), continuing from cap_in (the carried
        sponge capacity / Blake2s chaining value after cols_before columns) when given."""
        c, m = lde.shape
        if self.hasher == "poseidon2":
            call("bj_merkle_leaves_partial_d", lde.data_ptr(), c, lde.stride(0), m,
                 None if cap_in is None else cap_in.data_ptr(), out.data_ptr(), 1 if final else 0, stream_of(out))
        elif self.hasher == "blake2s":
            call("bj_blake2s_leaves_partial_d", lde.data_ptr(), c, lde.stride(0), m, cols_before,
                 None if cap_in is None else cap_in.data_ptr(), out.data_ptr(), 1 if final else 0, stream_of(out))
        else:
            if cap_in is not None or not final:
                raise ValueError("%s leaves cannot be continued over column ranges" % self.hasher)
            call(self._leaves_fn, lde.data_ptr(), c, lde.stride(0), m, out.data_ptr(), stream_of(out))

    def nodes(self, leaves, cap_size, out):
        call(self._nodes_fn, leaves.data_ptr(), leaves.shape[0], cap_size, out.data_ptr(), stream_of(out))

    def synthetic(self, out, log_n, first_col):
        call("bj_fill_synthetic_d", out.data_ptr(), out.shape[0], out.stride(0), log_n, 42, first_col,
             stream_of(out))


class _Done:
    def wait(self):
        pass


def _all_gather(out, inp, group=None, async_op=False):
    """out (G*k, ...) <- concat over ranks of inp (k, ...). RCCL (backend "nccl") runs in
    place on device memory and, with async_op, returns a handle whose wait() orders the
    current stream after it. gloo (the CPU tests) stages through the host synchronously."""
    import torch.distributed as dist
    if dist.get_backend(group) == "nccl":
        w = dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op)
        return w if async_op else None
    world = dist.get_world_size(group)
    src = inp.detach().cpu().contiguous()
    parts = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(parts, src, group=group)
    out.copy_(torch.cat(parts, 0).to(out.device))
    return _Done() if async_op else None


def _all_to_all(out, inp, group=None, async_op=False):
    """out (G*k, ...) <- block r of out is block `rank` of rank r's inp (G*k, ...). RCCL runs it on
    device memory (async handle as in _all_gather); gloo stages through the host."""
    import torch.distributed as dist
    if dist.get_backend(group) == "nccl":
        w = dist.all_to_all_single(out, inp, group=group, async_op=async_op)
        return w if async_op else None
    src = inp.detach().cpu().contiguous()
    dst = torch.empty_like(src)
    dist.all_to_all_single(dst, src, group=group)
    out.copy_(dst.to(out.device))
    return _Done() if async_op else None


class _NoTimer:
    def start(self, name):
        pass

    def stop(self, name):
        pass


class ShardedWorkspace:
    """Per-rank HBM buffers of a G-way sharded commit of C x 2^log_n at LDE 2^log_lde.

    G <= D (or fold_exchange False):
    coeffs (C, n)             all columns' coefficients (this rank's slices written locally)
    work   (K, m) | None      fold scratch, K = columns per chunk (G > D only)
    G > D with fold_exchange (the default):
    own    (C/G, n)           this rank's coefficients
    send   (C/G * G * m)      its columns folded for every rank, (G, c_k, m) per chunk
    folded (C, m)             every column folded for this rank (the all-to-all output)
    lde    (C, m)             this rank's leaf range of every column's LDE, m = n*D/G
    state  (m, 4) | None      carried sponge capacity between column chunks
    leaves (m, 4), nodes (m - cap_local, 4), cap (cap, 4)
    """

    def __init__(self, n_cols, log_n, log_lde, cap_size, rank, world, device="cuda", group=None, ops=None,
                 max_chunk_cols=MAX_CHUNK_COLS, fold_exchange=True, hasher="poseidon2"):
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
        self.ops = ops if ops is not None else HipShardOps(hasher)
        self.hasher = getattr(self.ops, "hasher", hasher)
        n = 1 << log_n
        self.m = m = (n << log_lde) >> log_g
        self.cols_per_rank = n_cols // world
        self.cap_local = max(1, cap_size // world)
        if m <= self.cap_local:
            raise ValueError("each shard needs more leaves than its cap slice")
        # column pipeline geometry
        unit = _chunk_unit(world)
        self.pipelined = self.cols_per_rank % unit == 0 and self.hasher in PARTIAL_HASHERS
        if self.pipelined:
            self.schedule = _chunk_schedule(self.cols_per_rank, unit, max_chunk_cols)
        else:
            self.schedule = [self.cols_per_rank]
        self.n_chunks = len(self.schedule)
        self.chunk_cols = world * max(self.schedule)
        kw = dict(dtype=torch.int64, device=device)
        self.fold_exchange = bool(fold_exchange) and log_g > log_lde
        if self.fold_exchange:
            self.coeffs = self.work = None
            self.own = torch.empty((self.cols_per_rank, n), **kw)
            self.send = torch.empty((self.cols_per_rank * world * m,), **kw)
            self.folded = torch.empty((n_cols, m), **kw)
        else:
            self.own = self.send = self.folded = None
            self.coeffs = torch.empty((n_cols, n), **kw)
            self.work = torch.empty((self.chunk_cols, m), **kw) if log_g > log_lde else None
        self.lde = torch.empty((n_cols, m), **kw)
        self.state = torch.empty((m, 4), **kw) if self.n_chunks > 1 else None
        self.leaves = torch.empty((m, 4), **kw)
        self.nodes = torch.empty((m - self.cap_local, 4), **kw)
        self.cap = torch.empty((cap_size, 4), **kw)
        if cap_size < world:
            self.roots = torch.empty((world, 4), **kw)
            self.top_nodes = torch.empty((world - cap_size, 4), **kw)
        if hasattr(self.ops, "prepare"):
            self.ops.prepare(log_n)
        elif self.lde.is_cuda:
            call("bj_prepare", log_n)

    def column_runs(self):
        """This rank's columns as (local_first, global_first, count) runs, one per chunk, in
        local order.  Chunk k (c_k columns per rank) covers global columns
        [G S_k, G (S_k + c_k)), S_k = sum of the earlier c; rank P owns its P-th c_k slice."""
        P = self.rank
        if not self.pipelined:
            return [(0, P * self.cols_per_rank, self.cols_per_rank)]
        runs, S = [], 0
        for c in self.schedule:
            runs.append((S, S * self.world + P * c, c))
            S += c
        return runs

    def chunk_columns(self, k):
        """Global column range [lo, hi) of chunk k."""
        if not self.pipelined:
            return 0, self.n_cols
        S = sum(self.schedule[:k])
        return self.world * S, self.world * (S + self.schedule[k])

    def send_chunk(self, lo, c):
        """(G, c, m) view of the send buffer for the run of c local columns starting at lo."""
        base = self.world * self.m * lo
        return self.send[base: base + self.world * c * self.m].view(self.world, c, self.m)

    @property
    def my_columns(self):
        return [g + i for _, g, c in self.column_runs() for i in range(c)]

    @property
    def leaf_range(self):
        return self.rank * self.m, (self.rank + 1) * self.m

    def synthetic_trace_shard(self):
        """This rank's columns of the synthetic trace, generated in place."""
        t = torch.empty((self.cols_per_rank, 1 << self.log_n), dtype=torch.int64, device=self.lde.device)
        for lo, g, c in self.column_runs():
            self.ops.synthetic(t[lo:lo + c], self.log_n, g)
        return t


def sharded_witness_commit(trace_shard, ws, timer=None):
    """Commit this rank's column shard (C/G, n; columns in ws.my_columns order) into `ws`.
    Collective over ws.group.

    `timer`, if given, has start(name) / stop(name) called around the compute steps
    ("ifft", "lde", "leaves", "nodes"); the bench records events there."""
    ops = ws.ops
    timer = timer or _NoTimer()
    if tuple(trace_shard.shape) != (ws.cols_per_rank, 1 << ws.log_n):
        raise ValueError("trace shard must be (%d, %d)" % (ws.cols_per_rank, 1 << ws.log_n))
    runs = ws.column_runs()
    handles = []
    # chunk k's all-gather is issued as soon as this rank's part of it is transformed, so it
    # overlaps the transforms of the later chunks
    for k, (lo, g, c) in enumerate(runs):
        c0, c1 = ws.chunk_columns(k)
        if ws.fold_exchange:
            # fold this rank's chunk columns for every rank, then one all-to-all
            send = ws.send_chunk(lo, c)
            timer.start("ifft")
            ops.coeffs(trace_shard[lo:lo + c], ws.own[lo:lo + c], ws.log_n)
            ops.fold_shards(ws.own[lo:lo + c], ws.log_n, ws.log_lde, ws.log_g, send)
            timer.stop("ifft")
            # (fold_exchange implies G > D >= 2)
            handles.append(_all_to_all(ws.folded[c0:c1], send.view(ws.world * c, ws.m), ws.group, async_op=True))
            continue
        timer.start("ifft")
        ops.coeffs(trace_shard[lo:lo + c], ws.coeffs[g:g + c], ws.log_n)
        timer.stop("ifft")
        if ws.world > 1:
            handles.append(_all_gather(ws.coeffs[c0:c1], ws.coeffs[g:g + c], ws.group, async_op=True))
        else:
            handles.append(_Done())
    for k in range(ws.n_chunks):
        handles[k].wait()
        c0, c1 = ws.chunk_columns(k)
        cols = slice(c0, c1)
        timer.start("lde")
        if ws.fold_exchange:
            ops.lde_shard_folded(ws.folded[cols], ws.log_n, ws.log_lde, ws.log_g, ws.rank, ws.lde[cols])
        else:
            work = None if ws.work is None else ws.work[:c1 - c0]
            ops.lde_shard(ws.coeffs[cols], ws.log_n, ws.log_lde, ws.log_g, ws.rank, work, ws.lde[cols])
        timer.stop("lde")
        last = k == ws.n_chunks - 1
        timer.start("leaves")
        ops.leaves(ws.lde[cols], ws.leaves if last else ws.state, cap_in=None if k == 0 else ws.state, final=last,
                   cols_before=c0)
        timer.stop("leaves")
    timer.start("nodes")
    ops.nodes(ws.leaves, ws.cap_local, ws.nodes)
    timer.stop("nodes")
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
    return ws


def _subtree_level(leaves, nodes, n_leaves, level):
    """Level `level` (0 = leaves) of a tree stored as leaves + concatenated node levels."""
    if level == 0:
        return leaves
    off, ln = 0, n_leaves
    for _ in range(level - 1):
        ln //= 2
        off += ln
    return nodes[off: off + ln // 2]


def sharded_query(ws, tree_idx):
    """OracleQuery::construct (proof.rs:65-97) for a one-element-per-column leaf over a sharded
    commit: leaf_elements = every column's LDE value at flat leaf index tree_idx (coset * n +
    row), proof = MerkleTreeWithCap::get_proof (merkle_tree.rs:462-480) of the global tree.
    The owning rank reads its row and its subtree path; when cap < G the replicated top levels
    (gathered roots) finish the path. Collective over ws.group: every rank returns the same
    (leaf_elements (C,), leaf_hash (4,), proof (depth, 4)) as host int64 tensors."""
    import torch.distributed as dist
    nl = ws.m * ws.world
    if not 0 <= tree_idx < nl:
        raise ValueError("tree index out of range")
    owner, local = divmod(tree_idx, ws.m)
    local_depth = _log2(ws.m) - _log2(ws.cap_local)
    top_depth = _log2(ws.world) - _log2(ws.cap_size) if ws.cap_size < ws.world else 0
    size = ws.n_cols + 4 + 4 * (local_depth + top_depth)
    buf = torch.zeros(size, dtype=torch.int64, device=ws.lde.device)
    if ws.rank == owner:
        parts = [ws.lde[:, local], ws.leaves[local]]
        idx = local
        for lvl in range(local_depth):
            parts.append(_subtree_level(ws.leaves, ws.nodes, ws.m, lvl)[idx ^ 1])
            idx >>= 1
        buf.copy_(torch.cat([p.reshape(-1) for p in parts] + [torch.zeros(4 * top_depth, dtype=torch.int64,
                                                                          device=buf.device)]))
    if top_depth:
        # the top tree over the G subtree roots is replicated on every rank
        idx = owner
        tops = []
        for lvl in range(top_depth):
            tops.append(_subtree_level(ws.roots, ws.top_nodes, ws.world, lvl)[idx ^ 1])
            idx >>= 1
        buf[size - 4 * top_depth:] = torch.cat([t.reshape(-1) for t in tops])
    if ws.world > 1:
        if dist.get_backend(ws.group) == "nccl":
            dist.broadcast(buf, src=owner, group=ws.group)
        else:
            host = buf.cpu()
            dist.broadcast(host, src=owner, group=ws.group)
            buf = host
    buf = buf.cpu()
    c = ws.n_cols
    return buf[:c], buf[c:c + 4], buf[c + 4:].reshape(-1, 4)


# ------------------------------------------------------------------ native collective commit
HASHER_IDS = {"poseidon2": 0, "blake2s": 1, "keccak256": 2}


def native_columns(n_cols, world, rank, hasher="poseidon2"):
    """bj_sharded_columns: the global trace columns rank `rank` of `world` holds, in the order of
    its trace-shard rows (the same deal as ShardedWorkspace.my_columns, except that at G = 1 the
    native commit runs one chunk).  Host logic only."""
    import ctypes
    from ._lib import load, check
    log_g = _log2(world)
    out = (ctypes.c_uint32 * (n_cols // world if n_cols % world == 0 and n_cols else 1))()
    check(load().bj_sharded_columns(n_cols, log_g, rank, HASHER_IDS[hasher], out), "bj_sharded_columns")
    return list(out)


class LocalGroup:
    """bj_comm_local_group_*: in-process ranks (threads) sharing one device.  A rehearsal
    transport that runs the native pipeline multi-rank on one GPU; not for performance."""

    def __init__(self, world):
        import ctypes
        from ._lib import load, check
        h = ctypes.c_void_p()
        check(load().bj_comm_local_group_create(world, ctypes.byref(h)), "bj_comm_local_group_create")
        self.handle, self.world = h, world

    def comm(self, rank):
        return NativeComm._make("bj_comm_init_local", self.handle, rank, world=self.world, rank=rank, keep=self)

    def close(self):
        from ._lib import load
        if self.handle:
            load().bj_comm_local_group_destroy(self.handle)
            self.handle = None


class NativeComm:
    """An opaque bj_comm (include/boojum_mi355x.h): the communicator of bj_sharded_commit_d."""

    def __init__(self, handle, world, rank, keep=None):
        self.handle, self.world, self.rank, self._keep = handle, world, rank, keep

    @classmethod
    def _make(cls, fn, *args, world, rank, keep=None):
        import ctypes
        from ._lib import load, check
        h = ctypes.c_void_p()
        check(getattr(load(), fn)(*args, ctypes.byref(h)), fn)
        return cls(h, world, rank, keep)

    @classmethod
    def rccl(cls, group=None):
        """A fresh RCCL communicator over the ranks of the torch.distributed group (one process
        per GPU, current device): rank 0 makes the unique id, the group broadcasts it, every rank
        joins (ncclCommInitRank).  Collective."""
        import ctypes
        import torch.distributed as dist
        from ._lib import load, check
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        uid = (ctypes.c_uint8 * 128)()
        if rank == 0:
            check(load().bj_comm_rccl_unique_id(uid), "bj_comm_rccl_unique_id")
        box = [bytes(uid)]
        dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        uid = (ctypes.c_uint8 * 128).from_buffer_copy(box[0])
        return cls._make("bj_comm_init_rccl", uid, world, rank, world=world, rank=rank)

    def close(self):
        from ._lib import load
        if self.handle:
            load().bj_comm_destroy(self.handle)
            self.handle = None


class NativeShardedResult:
    """Rank P's outputs of bj_sharded_commit_d: lde (C, m), leaves (m, 4), nodes
    (m - cap_local, 4), cap (cap, 4), all int64 on the device."""

    def __init__(self, n_cols, log_n, log_lde, cap_size, world, device="cuda"):
        m = ((1 << log_n) << log_lde) // world
        cap_local = max(1, cap_size // world)
        kw = dict(dtype=torch.int64, device=device)
        self.m, self.cap_local = m, cap_local
        self.lde = torch.empty((n_cols, m), **kw)
        self.leaves = torch.empty((m, 4), **kw)
        self.nodes = torch.empty((m - cap_local, 4), **kw)
        self.cap = torch.empty((cap_size, 4), **kw)


def native_sharded_commit(comm, trace_shard, n_cols, log_n, log_lde, cap_size, hasher="poseidon2", out=None):
    """bj_sharded_commit_d on the current stream: this rank's part of the G-way witness commit,
    trace_shard (C/G, n) in native_columns order.  Collective over `comm`."""
    if tuple(trace_shard.shape) != (n_cols // comm.world, 1 << log_n) or trace_shard.stride(1) != 1:
        raise ValueError("trace shard must be (%d, %d) with unit-stride rows" % (n_cols // comm.world, 1 << log_n))
    out = out or NativeShardedResult(n_cols, log_n, log_lde, cap_size, comm.world, trace_shard.device)
    call("bj_sharded_commit_d", comm.handle, trace_shard.data_ptr(), trace_shard.stride(0), n_cols, log_n, log_lde,
         cap_size, HASHER_IDS[hasher], out.lde.data_ptr(), out.leaves.data_ptr(), out.nodes.data_ptr(),
         out.cap.data_ptr(), stream_of(out.lde))
    return out


def native_sharded_query(comm, res, n_cols, log_n, log_lde, cap_size, tree_idx, hasher="poseidon2"):
    """bj_sharded_query_h: OracleQuery::construct on a native sharded commit (res is this rank's
    NativeShardedResult).  Collective over `comm`; every rank returns the same
    (leaf_elements (C,), leaf_hash (4,), proof (depth, 4)) as numpy uint64."""
    import ctypes
    import numpy as np
    depth = (log_n + log_lde) - _log2(cap_size)
    elems = np.zeros(n_cols, dtype=np.uint64)
    leaf = np.zeros(4, dtype=np.uint64)
    proof = np.zeros((max(depth, 1), 4), dtype=np.uint64)
    p = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))  # noqa: E731
    call("bj_sharded_query_h", comm.handle, res.lde.data_ptr(), res.leaves.data_ptr(), res.nodes.data_ptr(), n_cols,
         log_n, log_lde, cap_size, HASHER_IDS[hasher], tree_idx, p(elems), p(leaf), p(proof), stream_of(res.lde))
    return elems, leaf, proof[:depth]
