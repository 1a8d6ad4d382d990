"""CPU model of the native collective commit (csrc/collective.hip, bj_sharded_commit_d) -- TEST ONLY.

The product runs the G-way commit as one native call per rank.  This module restates its
schedule in Python over torch.distributed (gloo) with the oracle's CPU steps
(shard_cpu_ops.CpuShardOps), so the multi-process tests can check, without a GPU, the
partition math the native call implements:

  * the column deal (chunk k = G c_k consecutive columns, rank P the P-th run of c_k,
    u = 8 / gcd(8, G), c = u, u, then x3/2 (G <= 4) or x2 (G >= 8) rounded down to u but at
    least u more, capped at 32; one contiguous chunk otherwise) --
    compared with bj_sharded_columns by tests/test_native_columns.py;
  * the LDE at D = 2^log_lde committed over its first k = 2^log_k cosets (prover.rs:313-347):
    rank P owns leaf range [P m, (P+1) m), m = k n / G, and the same range of every block of k
    cosets, i.e. range j G + P of the D-coset domain cut into 2^ls ranges, ls = log G + log D -
    log k; its LDE is (B, C, m), B = D / k;
  * the exchange: G <= D all-gather of the coefficients, then each rank's ranges (folded at the
    receiver when G > k); G > D the sender folds its columns for every (block, rank) and one
    all-to-all per block delivers them;
  * the sponge carried across column chunks, the subtree, and the cap (cap < G: the G subtree
    roots gathered and the top levels hashed on every rank); openings (bj_sharded_query_h).
"""
import math

import torch
import torch.distributed as dist

MAX_CHUNK_COLS = 32
PARTIAL_HASHERS = ("poseidon2", "blake2s")


def _log2(n):
    if n <= 0 or n & (n - 1):
        raise ValueError("size must be a power of two, got %d" % n)
    return n.bit_length() - 1


def chunk_unit(world):
    return 8 // math.gcd(8, world)


def chunk_schedule(cols_per_rank, unit, max_cols=MAX_CHUNK_COLS, world=8):
    max_cols = max(unit, max_cols // unit * unit)
    sched, done, b = [], 0, unit
    while done < cols_per_rank:
        take = min(b, cols_per_rank - done)
        sched.append(take)
        done += take
        if len(sched) >= 2:
            b = min(max(b + unit, b * 3 // 2 // unit * unit) if world <= 4 else 2 * b, max_cols)
    return sched


def _all_gather(out, inp, group=None):
    world = dist.get_world_size(group)
    parts = [torch.empty_like(inp) for _ in range(world)]
    dist.all_gather(parts, inp.contiguous(), group=group)
    out.copy_(torch.cat(parts, 0))


def _all_to_all(out, inp, group=None):
    dst = torch.empty_like(inp)
    dist.all_to_all_single(dst, inp.contiguous(), group=group)
    out.copy_(dst)


class ShardModel:
    """Per-rank buffers and geometry of a G-way commit of C x 2^log_n at LDE 2^log_lde over the
    first 2^log_k cosets (default all)."""

    def __init__(self, n_cols, log_n, log_lde, cap_size, rank, world, ops, log_k=None, max_chunk_cols=MAX_CHUNK_COLS,
                 fold_exchange=True, hasher="poseidon2", group=None):
        log_k = log_lde if log_k is None else log_k
        log_g = _log2(world)
        _log2(cap_size)
        if n_cols % world:
            raise ValueError("n_cols (%d) must be a multiple of the number of shards (%d)" % (n_cols, world))
        if log_lde == 0:
            raise ValueError("lde degree must be > 1 (utils.rs:283)")
        if not 0 <= log_k <= log_lde:
            raise ValueError("committed cosets exceed the lde degree")
        if log_g > log_n + log_k:
            raise ValueError("more shards than committed leaves")
        if cap_size >= (1 << (log_n + log_k)):
            raise ValueError("tree size must exceed cap size")
        self.n_cols, self.log_n, self.log_lde, self.log_k, self.cap_size = n_cols, log_n, log_lde, log_k, cap_size
        self.rank, self.world, self.log_g, self.group, self.ops, self.hasher = rank, world, log_g, group, ops, hasher
        n = 1 << log_n
        self.m = m = (n << log_k) >> log_g
        self.blocks = 1 << (log_lde - log_k)
        self.ls = log_g + log_lde - log_k
        self.cols_per_rank = n_cols // world
        self.cap_local = max(1, cap_size // world)
        if m <= self.cap_local:
            raise ValueError("each shard needs more leaves than its cap slice")
        unit = chunk_unit(world)
        self.pipelined = world > 1 and self.cols_per_rank % unit == 0 and hasher in PARTIAL_HASHERS
        self.schedule = chunk_schedule(self.cols_per_rank, unit, max_chunk_cols, world) if self.pipelined \
            else [self.cols_per_rank]
        self.n_chunks = len(self.schedule)
        self.fold_exchange = bool(fold_exchange) and log_g > log_lde
        kw = dict(dtype=torch.int64)
        B = self.blocks
        if self.fold_exchange:
            self.own = torch.empty((self.cols_per_rank, n), **kw)
            self.folded = torch.empty((B, n_cols, m), **kw)
        else:
            self.coeffs = torch.empty((n_cols, n), **kw)
        self.lde = torch.empty((B, n_cols, m), **kw)
        self.state = torch.empty((m, 4), **kw) if self.n_chunks > 1 else None
        self.leaves = torch.empty((m, 4), **kw)
        self.nodes = torch.empty((m - self.cap_local, 4), **kw)
        self.cap = torch.empty((cap_size, 4), **kw)
        if cap_size < world:
            self.roots = torch.empty((world, 4), **kw)
            self.top_nodes = torch.empty((world - cap_size, 4), **kw)

    def column_runs(self):
        """(local_first, global_first, count) per chunk."""
        P = self.rank
        if not self.pipelined:
            return [(0, P * self.cols_per_rank, self.cols_per_rank)]
        runs, S = [], 0
        for c in self.schedule:
            runs.append((S, S * self.world + P * c, c))
            S += c
        return runs

    def chunk_columns(self, k):
        if not self.pipelined:
            return 0, self.n_cols
        S = sum(self.schedule[:k])
        return self.world * S, self.world * (S + self.schedule[k])

    @property
    def my_columns(self):
        return [g + i for _, g, c in self.column_runs() for i in range(c)]

    def synthetic_trace_shard(self):
        t = torch.empty((self.cols_per_rank, 1 << self.log_n), dtype=torch.int64)
        for lo, g, c in self.column_runs():
            self.ops.synthetic(t[lo:lo + c], self.log_n, g)
        return t


def commit(trace_shard, ws):
    """The schedule of bj_sharded_commit_d on this rank (collective over ws.group)."""
    ops, G, P, B = ws.ops, ws.world, ws.rank, ws.blocks
    runs = ws.column_runs()
    for k, (lo, g, c) in enumerate(runs):
        c0, c1 = ws.chunk_columns(k)
        if ws.fold_exchange:
            ops.coeffs(trace_shard[lo:lo + c], ws.own[lo:lo + c], ws.log_n)
            for j in range(B):
                send = torch.empty((G, c, ws.m), dtype=torch.int64)
                ops.fold_shards(ws.own[lo:lo + c], ws.log_n, ws.log_lde, ws.ls, send, shards=range(j * G, j * G + G))
                _all_to_all(ws.folded[j, c0:c1], send.view(G * c, ws.m), ws.group)
        else:
            ops.coeffs(trace_shard[lo:lo + c], ws.coeffs[g:g + c], ws.log_n)
            if G > 1:
                _all_gather(ws.coeffs[c0:c1], ws.coeffs[g:g + c], ws.group)
    for k in range(ws.n_chunks):
        c0, c1 = ws.chunk_columns(k)
        for j in range(B):
            out = ws.lde[j, c0:c1]
            if ws.fold_exchange:
                ops.lde_shard_folded(ws.folded[j, c0:c1], ws.log_n, ws.log_lde, ws.ls, j * G + P, out)
            else:
                ops.lde_shard(ws.coeffs[c0:c1], ws.log_n, ws.log_lde, ws.ls, j * G + P, None, out)
        last = k == ws.n_chunks - 1
        ops.leaves(ws.lde[0, c0:c1], ws.leaves if last else ws.state, cap_in=None if k == 0 else ws.state,
                   final=last, cols_before=c0)
    ops.nodes(ws.leaves, ws.cap_local, ws.nodes)
    local_cap = ws.nodes[-ws.cap_local:]
    if ws.cap_size >= G:
        if G > 1:
            _all_gather(ws.cap, local_cap, ws.group)
        else:
            ws.cap.copy_(local_cap)
    else:
        _all_gather(ws.roots, local_cap, ws.group)
        ops.nodes(ws.roots, ws.cap_size, ws.top_nodes)
        ws.cap.copy_(ws.top_nodes[-ws.cap_size:])
    return ws


def _level(leaves, nodes, n_leaves, level):
    if level == 0:
        return leaves
    off, ln = 0, n_leaves
    for _ in range(level - 1):
        ln //= 2
        off += ln
    return nodes[off: off + ln // 2]


def query(ws, tree_idx):
    """bj_sharded_query_h: (leaf_elements (C,), leaf_hash (4,), proof (depth, 4)) on every rank."""
    nl = ws.m * ws.world
    if not 0 <= tree_idx < nl:
        raise ValueError("tree index out of range")
    owner, local = divmod(tree_idx, ws.m)
    local_depth = _log2(ws.m) - _log2(ws.cap_local)
    top_depth = _log2(ws.world) - _log2(ws.cap_size) if ws.cap_size < ws.world else 0
    size = ws.n_cols + 4 + 4 * (local_depth + top_depth)
    buf = torch.zeros(size, dtype=torch.int64)
    if ws.rank == owner:
        parts = [ws.lde[0, :, local], ws.leaves[local]]
        idx = local
        for lvl in range(local_depth):
            parts.append(_level(ws.leaves, ws.nodes, ws.m, lvl)[idx ^ 1])
            idx >>= 1
        buf[:size - 4 * top_depth] = torch.cat([p.reshape(-1) for p in parts])
    if top_depth:
        idx, tops = owner, []
        for lvl in range(top_depth):
            tops.append(_level(ws.roots, ws.top_nodes, ws.world, lvl)[idx ^ 1])
            idx >>= 1
        buf[size - 4 * top_depth:] = torch.cat([t.reshape(-1) for t in tops])
    if ws.world > 1:
        dist.broadcast(buf, src=owner, group=ws.group)
    c = ws.n_cols
    return buf[:c], buf[c:c + 4], buf[c + 4:].reshape(-1, 4)
