#!/usr/bin/env python3
"""Per-rank compute of the G-way sharded commit, measured on one GPU with the exchange
stubbed out: rank P's LDE range, leaves and subtree for G = 1, 2, 4, 8 at C3.  The result
bounds the multi-GPU step time from below (exchange fully hidden).  It is not a bench
line (the coefficient buffer holds this rank's own columns only, so the values are not a
real commit).

usage: python tools/shard_compute_probe.py [config]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "era-boojum_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from boojum_amd import sharded
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
    n_cols, log_n, log_lde, cap = bench.CONFIGS[cfg]
    out = {}

    def compute(ws, tr):
        """sharded_witness_commit without its collectives (rank 0's compute only)."""
        ops = ws.ops
        for k, (lo, g, c) in enumerate(ws.column_runs()):
            if ws.fold_exchange:
                ops.coeffs(tr[lo:lo + c], ws.own[lo:lo + c], ws.log_n)
                ops.fold_shards(ws.own[lo:lo + c], ws.log_n, ws.log_lde, ws.log_g, ws.send_chunk(lo, c))
            else:
                ops.coeffs(tr[lo:lo + c], ws.coeffs[g:g + c], ws.log_n)
        for k in range(ws.n_chunks):
            c0, c1 = ws.chunk_columns(k)
            if ws.fold_exchange:
                ops.lde_shard_folded(ws.folded[c0:c1], ws.log_n, ws.log_lde, ws.log_g, ws.rank, ws.lde[c0:c1])
            else:
                work = None if ws.work is None else ws.work[:c1 - c0]
                ops.lde_shard(ws.coeffs[c0:c1], ws.log_n, ws.log_lde, ws.log_g, ws.rank, work, ws.lde[c0:c1])
            last = k == ws.n_chunks - 1
            ops.leaves(ws.lde[c0:c1], ws.leaves if last else ws.state, cap_in=None if k == 0 else ws.state,
                       final=last)
        ops.nodes(ws.leaves, ws.cap_local, ws.nodes)

    class TimedOps:
        """Wraps the ops object: events around every call, summed per op name."""

        def __init__(self, inner):
            self.inner, self.ev = inner, []

        def __getattr__(self, name):
            fn = getattr(self.inner, name)
            if not callable(fn):
                return fn

            def run(*a, **k):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                r = fn(*a, **k)
                e.record()
                self.ev.append((name, s, e))
                return r
            return run

        def totals(self, reps):
            torch.cuda.synchronize()
            acc = {}
            for name, s, e in self.ev:
                acc[name] = acc.get(name, 0.0) + s.elapsed_time(e)
            return {k: round(v / reps, 3) for k, v in acc.items()}

    runs = [(w, True) for w in (1, 2, 4, 8)] + [(w, False) for w in (8,) if w > (1 << log_lde)]
    for world, fold in runs:
        ws = sharded.ShardedWorkspace(n_cols, log_n, log_lde, cap, 0, world, device="cuda", fold_exchange=fold)
        tr = ws.synthetic_trace_shard()
        compute(ws, tr)   # warm-up
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(3):
            compute(ws, tr)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 3
        timed = TimedOps(ws.ops)
        ws.ops = timed
        compute(ws, tr)
        phases = timed.totals(1)
        ws.ops = timed.inner
        out["%d%s" % (world, "" if fold or world <= (1 << log_lde) else "_allgather")] = {
            "ms_per_rank": round(ms, 2), "chunks": ws.n_chunks,
            "ideal_elems_per_s": n_cols * (1 << log_n) / (ms * 1e-3), "phase_ms": phases}
        del ws, tr
        torch.cuda.empty_cache()
    print(json.dumps({"config": cfg, "per_rank_compute": out}))


if __name__ == "__main__":
    main()
