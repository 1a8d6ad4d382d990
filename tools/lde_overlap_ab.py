#!/usr/bin/env python3
"""Same-box A/B of the three-pass LDE (bj_lde_ex_d, C3 by default) with the middle and final
passes overlapped by column chunk (BJ_LDE_OVERLAP=c: chunk k's middle pass on the caller's
stream, its final pass on a second stream behind an event; a chunk written "64h" also runs the
inverse head by chunk on a third stream, BJ_LDE_OVERLAP_HEAD=1) against the plain order
(BJ_LDE_OVERLAP=0).  Variants alternate in rounds; every variant's LDE must equal the plain
one's bit for bit.  Prints one JSON line per variant (ms per LDE, median over rounds).

usage: python tools/lde_overlap_ab.py [config] [rounds] [reps] [chunk ...]
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "era-boojum_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from boojum_amd import commit
    from boojum_amd._lib import call
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    chunks = sys.argv[4:] or ["0", "128", "64", "32"]
    n_cols, log_n, log_lde, _ = bench.CONFIGS[cfg]
    n, D = 1 << log_n, 1 << log_lde
    trace = commit.synthetic_trace(n_cols, log_n)
    scratch = torch.empty((n_cols, n), dtype=torch.int64, device="cuda")
    lde = torch.empty((n_cols, D, n), dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream

    def run():
        call("bj_lde_ex_d", trace.data_ptr(), n_cols, n, log_n, log_lde, scratch.data_ptr(), lde.data_ptr(), 0, st)

    os.environ["BJ_LDE_OVERLAP"] = "0"
    run()
    torch.cuda.synchronize()
    ref = lde.clone()
    times = {c: [] for c in chunks}
    for r in range(rounds):
        for c in chunks:
            os.environ["BJ_LDE_OVERLAP"] = c.rstrip("h")
            os.environ["BJ_LDE_OVERLAP_HEAD"] = "1" if c.endswith("h") else "0"
            lde.zero_()
            run()
            run()
            torch.cuda.synchronize()
            assert torch.equal(lde, ref), "chunk %s: LDE differs from the plain order" % c
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            times[c].append(e0.elapsed_time(e1) / reps)
            print("round %d chunk %4s %.2f ms" % (r, c, times[c][-1]), flush=True)
    os.environ["BJ_LDE_OVERLAP"] = "0"
    for c in chunks:
        print(json.dumps({"config": cfg, "chunk_cols": int(c.rstrip("h")), "head_chunked": c.endswith("h"),
                          "ms_per_lde": statistics.median(times[c]),
                          "all": [round(t, 2) for t in times[c]]}), flush=True)


if __name__ == "__main__":
    main()
