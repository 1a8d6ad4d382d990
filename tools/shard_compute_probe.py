#!/usr/bin/env python3
"""Per-rank compute of the G-way sharded commit, measured on one GPU with the exchange stubbed
out: rank 0 runs the native collective call (bj_sharded_commit_d) over a transport whose
exchanges move nothing (NativeComm.null), so the time is its iNTTs (+ folds), its LDE range,
leaves and subtree alone.  The result bounds the multi-GPU step time from below (exchange fully
hidden).  It is not a bench line: the received buffers are never filled, so the values are not
a commitment.

usage: python tools/shard_compute_probe.py [config ...]      (default: C3 at G = 1, 2, 4, 8 and
                                                               C4 at G = 8, one coset per rank)
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
    from boojum_amd._lib import call
    from boojum_amd.field import stream_of
    from boojum_amd.sharded import NativeComm, NativeShardedResult, native_columns, native_sharded_commit
    plan = [("C3", 1), ("C3", 2), ("C3", 4), ("C3", 8), ("C4", 8)]
    if len(sys.argv) > 1:
        plan = [(c, w) for c, w in plan if c in sys.argv[1:]]
    out = {}
    for cfg, world in plan:
        n_cols, log_n, log_lde, cap = bench.CONFIGS[cfg]
        n = 1 << log_n
        comm = NativeComm.null(world, 0) if world > 1 else NativeComm.rccl_world1()
        tr = torch.empty((n_cols // world, n), dtype=torch.int64, device="cuda")
        for j, c in enumerate(native_columns(n_cols, world, 0)):
            call("bj_fill_synthetic_d", tr[j].data_ptr(), 1, n, log_n, 42, c, stream_of(tr))
        res = NativeShardedResult(n_cols, log_n, log_lde, cap, world)
        native_sharded_commit(comm, tr, n_cols, log_n, log_lde, cap, out=res)   # warm-up
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 3
        s.record()
        for _ in range(reps):
            native_sharded_commit(comm, tr, n_cols, log_n, log_lde, cap, out=res)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / reps
        # the same calls once more with the phase events on (bj_comm_set_timing)
        comm.set_timing(True)
        for _ in range(reps):
            native_sharded_commit(comm, tr, n_cols, log_n, log_lde, cap, out=res)
        torch.cuda.synchronize()
        ph, calls = comm.phase_ms()
        comm.set_timing(False)
        recv = 0 if world == 1 else (
            8 * n_cols * ((n << log_lde) // world) * (world - 1) // world if world > (1 << log_lde)
            else 8 * n * n_cols * (world - 1) // world)
        interfered = None
        if recv and os.environ.get("PROBE_INTERFERE"):
            # the same calls while a second, high-priority stream copies `recv` bytes device to
            # device per call (what RCCL writes into this GPU's memory), to price the exchange's
            # contention for CUs and HBM when it overlaps the compute
            chunk = 256 << 20
            a_buf = torch.empty(chunk // 8, dtype=torch.int64, device="cuda")
            b_buf = torch.empty_like(a_buf)
            side = torch.cuda.Stream(priority=-1)
            s2, e2 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s2.record()
            for _ in range(reps):
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    for _ in range(max(1, recv // chunk)):
                        b_buf.copy_(a_buf)
                native_sharded_commit(comm, tr, n_cols, log_n, log_lde, cap, out=res)
                torch.cuda.current_stream().wait_stream(side)
            e2.record()
            torch.cuda.synchronize()
            interfered = round(s2.elapsed_time(e2) / reps, 2)
            del a_buf, b_buf
        out["%s_G%d" % (cfg, world)] = {
            "ms_with_concurrent_copy_of_received_bytes": interfered,
            "ms_per_rank": round(ms, 2), "ideal_elems_per_s": n_cols * n / (ms * 1e-3),
            "phase_ms": {k: round(v / max(1, calls), 2) for k, v in ph.items()},
            "exchange": "none" if world == 1 else ("all-to-all (sender fold)" if world > (1 << log_lde)
                                                   else "all-gather"),
            "received_bytes_per_rank": 0 if world == 1 else (
                8 * n_cols * ((n << log_lde) // world) * (world - 1) // world if world > (1 << log_lde)
                else 8 * n * n_cols * (world - 1) // world)}
        print(json.dumps({cfg + "_G%d" % world: out["%s_G%d" % (cfg, world)]}), flush=True)
        comm.close()
        del tr, res
        torch.cuda.empty_cache()
    print(json.dumps({"per_rank_compute": out}))


if __name__ == "__main__":
    main()
