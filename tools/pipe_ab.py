#!/usr/bin/env python3
"""Same-box A/B of the one-GPU commit orders (bj_lde_commit_ex_d, ABI 2.4):

  serial   the three LDE passes, then every leaf, then the node levels, on one stream;
  pipe     the coset pipeline: the final pass coset by coset, each coset's leaves on a second
           stream as soon as it is final, the node levels once all leaves are in;
  pipe+X   the same with an environment knob of the library (BJ_LEAF_W4=1: the 128-VGPR leaf
           kernel, two of whose waves fit beside one LDE wave on a SIMD; BJ_FINAL_LDS_PAD=b:
           b bytes more LDS per final-pass block, one block per CU).

Variants run in rounds, alternated, so clock drift hits all of them alike; every commit's cap
is checked against the golden cap.  Prints one JSON line per variant (ms per commit, the
median over rounds).

usage: python tools/pipe_ab.py [config] [rounds] [steps] [variant ...]
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "era-boojum_amd"))
sys.path.insert(0, ROOT)

VARIANTS = [
    ("serial", 2, {}),
    ("pipe", 4, {}),
    ("pipe+w4", 4, {"BJ_LEAF_W4": "1"}),
    ("pipe+pad16k", 4, {"BJ_FINAL_LDS_PAD": "16384"}),
    ("pipe+w4+pad16k", 4, {"BJ_LEAF_W4": "1", "BJ_FINAL_LDS_PAD": "16384"}),
    ("pipe+s2hi", 4, {"BJ_PIPE_PRIO": "-1"}),
    ("pipe+s2lo", 4, {"BJ_PIPE_PRIO": "1"}),
]


def main():
    import torch
    import bench
    from boojum_amd import commit
    from boojum_amd._lib import call
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    only = sys.argv[4:]
    variants = [v for v in VARIANTS if not only or v[0] in only]
    n_cols, log_n, log_lde, cap = bench.CONFIGS[cfg]
    n = 1 << log_n
    trace = commit.synthetic_trace(n_cols, log_n)
    ws = commit.CommitWorkspace(n_cols, log_n, log_lde, cap)
    want = bench.golden_cap(cfg, "poseidon2")
    st = torch.cuda.current_stream().cuda_stream

    def run(flags):
        call("bj_lde_commit_ex_d", trace.data_ptr(), n_cols, n, log_n, log_lde, log_lde, cap, ws.scratch.data_ptr(),
             ws.lde.data_ptr(), ws.leaves.data_ptr(), ws.nodes.data_ptr(), None, flags, st)

    times = {name: [] for name, _, _ in variants}
    for r in range(rounds):
        for name, flags, env in variants:
            for k, v in env.items():
                os.environ[k] = v
            try:
                run(flags)
                run(flags)
                torch.cuda.synchronize()
                if want is not None:
                    assert bench.cap_matches(ws.cap, want), "%s: cap differs from the golden cap" % name
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(steps):
                    run(flags)
                e1.record()
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1) / steps)
            finally:
                for k in env:
                    del os.environ[k]
            print("round %d %-16s %.2f ms" % (r, name, times[name][-1]), flush=True)
    for name, _, env in variants:
        print(json.dumps({"config": cfg, "variant": name, "env": env, "ms_per_commit": statistics.median(times[name]),
                          "all": [round(t, 2) for t in times[name]]}), flush=True)


if __name__ == "__main__":
    main()
