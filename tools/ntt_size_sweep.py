#!/usr/bin/env python3
"""LDE throughput across column lengths: bj_lde_d on C columns of 2^log_n rows at LDE x2,
for log_n from 2^16 to 2^25 (two coset-folded CT passes cover 2^13..2^23, three passes
2^24..2^26, the DIF network the rest).  Prints one JSON line per size: ms per LDE and LDE elements per second.

usage: python tools/ntt_size_sweep.py [total_log_elems (default 28)]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "era-boojum_amd"))


def main():
    import torch
    from boojum_amd import commit
    from boojum_amd._lib import call
    total = int(sys.argv[1]) if len(sys.argv) > 1 else 28
    for log_n in range(16, 26):
        n_cols = max(1, 1 << (total - log_n))
        n = 1 << log_n
        trace = commit.synthetic_trace(n_cols, log_n)
        scratch = torch.empty_like(trace)
        lde = torch.empty((n_cols, 2, n), dtype=torch.int64, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        call("bj_lde_d", trace.data_ptr(), n_cols, n, log_n, 1, scratch.data_ptr(), lde.data_ptr(), st)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(3):
            call("bj_lde_d", trace.data_ptr(), n_cols, n, log_n, 1, scratch.data_ptr(), lde.data_ptr(), st)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 3
        print(json.dumps({"log_n": log_n, "cols": n_cols, "ms": round(ms, 3),
                          "lde_elems_per_s": 2 * n * n_cols / (ms * 1e-3),
                          "path": "ct" if 13 <= log_n <= 23 else ("ct, 3 passes" if log_n <= 26 else "dif")}), flush=True)
        del trace, scratch, lde
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
