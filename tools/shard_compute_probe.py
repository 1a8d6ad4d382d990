#!/usr/bin/env python3
"""Per-rank compute of the G-way sharded commit, measured on one GPU with the exchange stubbed
out: rank 0 runs the native collective call (bj_sharded_commit_d) over a transport whose
exchanges move nothing (NativeComm.null), so the time is its iNTTs (+ folds), its LDE range,
leaves and subtree alone.  The result bounds the multi-GPU step time from below (exchange fully
hidden).  It is not a bench line: the received buffers are never filled, so the values are not
a commitment.

usage: python tools/shard_compute_probe.py [config[:G] ...] (default: C3 at G = 1, 2, 4, 8 and
                                                               C4 at G = 8, one coset per rank)
"""
import json
import os
import sys

# PROBE_INTERFERE=1: also the same calls beside an exchange-shaped disturbance (interference());
# PROBE_PHASE_EVENTS_TIMED=1 times those calls with the phase events on, as rounds 4-5 did;
# PROBE_LOG_K=k commits the first 2^k of the 2^log_lde cosets (k < D: at G > 2^k the sender folds
# by F = G / 2^k)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "era-boojum_amd"))
sys.path.insert(0, ROOT)


# per-rank xGMI ingress of the exchange at G ranks: the links toward the other ranks (one per
# peer on the 8-GPU node's full mesh, at most 7) at an effective per-link, per-direction rate
LINK_GBS = (64.0, 153.0)


def links(world):
    return min(world - 1, 7)


def _timed(comm, tr, res, n_cols, log_n, log_lde, cap, reps, phase_events_in_timed=False, log_k=None):
    """ms per call (events around it on the compute stream) and the phase split.  The timed calls
    run as a production call does, without the library's phase events (bj_comm_set_timing), and
    the phase split comes from `reps` further calls with them on; phase_events_in_timed=True
    times the calls that record the phases (round 4 and round 5's r5o tables were taken so)."""
    import torch
    from boojum_amd.sharded import native_sharded_commit
    native_sharded_commit(comm, tr, n_cols, log_n, log_lde, cap, out=res, log_commit_cosets=log_k)  # warm-up
    torch.cuda.synchronize()
    comm.phase_ms()

    def run(timing):
        comm.set_timing(timing)
        tot = 0.0
        for _ in range(reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            native_sharded_commit(comm, tr, n_cols, log_n, log_lde, cap, out=res, log_commit_cosets=log_k)
            e.record()
            torch.cuda.synchronize()
            tot += s.elapsed_time(e)
        comm.set_timing(False)
        return tot / reps

    ms = None if phase_events_in_timed else run(False)
    ms_ev = run(True)
    ph, calls = comm.phase_ms()
    return (ms_ev if ms is None else ms), {k: v / max(1, calls) for k, v in ph.items()}


def interference(comm0, tr, res, n_cols, log_n, log_lde, cap, world, recv, reps, ph0, calls0, log_k=None):
    """The same call with each exchange replaced by an RCCL-shaped stand-in: a device-mode callback
    transport (bj_comm_init_callback) whose exchange launches tools/paced_copy.hip on the stream
    the library hands it -- the communicator's high-priority exchange stream, where RCCL's kernels
    run -- moving the bytes this rank receives in that exchange, (G - 1) x the per-rank block, with
    `channels` workgroups resident for the whole copy (as RCCL's collective kernels are) at the
    rank's xGMI ingress rate, links(G) x LINK_GBS; "burst" is the same copy unpaced.  So the
    compute stream sees the exchange's CU residency, its HBM traffic and its duration, chunk by
    chunk, as the column pipeline issues them.  Per shape: ms per call, the delta against the
    stubbed exchange, and the per-phase deltas (inverse + fold, LDE, leaves, nodes); the rest of a
    delta is exchange the pipeline left exposed."""
    import ctypes
    import torch
    from boojum_amd._lib import EXCHANGE_FN
    from boojum_amd.sharded import NativeComm
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libpaced_copy.so"))
    lib.paced_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int,
                               ctypes.c_double, ctypes.c_void_p]
    ring = 512 << 20  # a 512 MiB ring: past the 256 MiB Infinity Cache, so the bytes reach HBM
    a_buf = torch.empty(ring // 8, dtype=torch.int64, device="cuda")
    b_buf = torch.empty_like(a_buf)
    ev = bool(os.environ.get("PROBE_PHASE_EVENTS_TIMED"))
    base_ms, base_ph = _timed(comm0, tr, res, n_cols, log_n, log_lde, cap, reps, ev, log_k)
    rows = {"phase_events_in_timed_calls": ev,
            "stubbed": {"ms": round(base_ms, 2), "phase_ms": {k: round(v, 2) for k, v in base_ph.items()}}}
    shapes = [("burst_32ch", 32, 0.0)]
    for per_link in LINK_GBS:
        for ch in (8, 16, 32):
            shapes.append(("paced_%dch_%dGBs" % (ch, links(world) * per_link), ch, links(world) * per_link))
    for name, ch, gbps in shapes:
        def exchange(user, kind, send, recv_p, nbytes, stream, ch=ch, gbps=gbps):
            moved = (world - 1) * nbytes
            return lib.paced_copy(a_buf.data_ptr(), b_buf.data_ptr(), ring, max(moved, 1 << 18), ch, gbps, stream)
        fn = EXCHANGE_FN(exchange)
        comm = NativeComm._make("bj_comm_init_callback", world, 0, fn, None, 0, world=world, rank=0, keep=fn)
        try:
            ms, ph = _timed(comm, tr, res, n_cols, log_n, log_lde, cap, reps, ev, log_k)
        finally:
            comm.close()
        rows[name] = {"ms": round(ms, 2), "delta_ms": round(ms - base_ms, 2),
                      "phase_delta_ms": {k: round(ph[k] - base_ph[k], 2) for k in ph},
                      "exposed_ms": round((ms - base_ms) - sum(ph[k] - base_ph[k] for k in ph), 2)}
    del a_buf, b_buf
    return rows


def main():
    import torch
    import bench
    from boojum_amd._lib import call
    from boojum_amd.field import stream_of
    from boojum_amd.sharded import NativeComm, NativeShardedResult, native_columns, native_sharded_commit
    plan = [("C3", 1), ("C3", 2), ("C3", 4), ("C3", 8), ("C4", 8)]
    if len(sys.argv) > 1:
        # "C3" selects every world of a config, "C3:8" one world
        plan = [(c, w) for c, w in plan if c in sys.argv[1:] or "%s:%d" % (c, w) in sys.argv[1:]]
    out = {}
    for cfg, world in plan:
        n_cols, log_n, log_lde, cap = bench.CONFIGS[cfg]
        log_k = int(os.environ.get("PROBE_LOG_K", log_lde))
        n = 1 << log_n
        comm = NativeComm.null(world, 0) if world > 1 else NativeComm.rccl_world1()
        tr = torch.empty((n_cols // world, n), dtype=torch.int64, device="cuda")
        for j, c in enumerate(native_columns(n_cols, world, 0)):
            call("bj_fill_synthetic_d", tr[j].data_ptr(), 1, n, log_n, 42, c, stream_of(tr))
        res = NativeShardedResult(n_cols, log_n, log_lde, cap, world, log_commit_cosets=log_k)
        native_sharded_commit(comm, tr, n_cols, log_n, log_lde, cap, out=res, log_commit_cosets=log_k)  # warm-up
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 3
        s.record()
        for _ in range(reps):
            native_sharded_commit(comm, tr, n_cols, log_n, log_lde, cap, out=res, log_commit_cosets=log_k)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / reps
        # the same calls once more with the phase events on (bj_comm_set_timing)
        comm.set_timing(True)
        for _ in range(reps):
            native_sharded_commit(comm, tr, n_cols, log_n, log_lde, cap, out=res, log_commit_cosets=log_k)
        torch.cuda.synchronize()
        ph, calls = comm.phase_ms()
        comm.set_timing(False)
        recv = 0 if world == 1 else (
            8 * n_cols * ((n << log_lde) // world) * (world - 1) // world if world > (1 << log_lde)
            else 8 * n * n_cols * (world - 1) // world)
        interfered = None
        if recv and os.environ.get("PROBE_INTERFERE"):
            interfered = interference(comm, tr, res, n_cols, log_n, log_lde, cap, world, recv, reps, ph, calls, log_k)
        out["%s_G%d" % (cfg, world)] = {
            "interference": interfered,
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
