"""Same-box A/B of the C3 LDE with and without the monomial write-back (bj_lde_d against
bj_lde_ex_d without BJ_LDE_KEEP_MONOMIALS), alternated, HIP events on the work stream; prints
one JSON line per variant and round, then the medians."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "era-boojum_amd"))


def main(rounds=6, reps=4, n_cols=256, log_n=22, log_d=2):
    import torch
    from boojum_amd import commit
    from boojum_amd._lib import call
    trace = commit.synthetic_trace(n_cols, log_n)
    n = 1 << log_n
    scratch = torch.empty((n_cols, n), dtype=torch.int64, device="cuda")
    lde = torch.empty((n_cols, 1 << log_d, n), dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    ref = None

    def run(keep):
        if keep:
            call("bj_lde_d", trace.data_ptr(), n_cols, n, log_n, log_d, scratch.data_ptr(), lde.data_ptr(), st)
        else:
            call("bj_lde_ex_d", trace.data_ptr(), n_cols, n, log_n, log_d, scratch.data_ptr(), lde.data_ptr(), 0, st)

    res = {True: [], False: []}
    for keep in (True, False):  # warm-up, and the two LDEs must agree
        run(keep)
        torch.cuda.synchronize()
        h = torch.sum(lde.view(-1)[:: 1 << 10]).item()
        ref = h if ref is None else ref
        assert h == ref, "LDE differs with and without the monomials"
    for r in range(rounds):
        for keep in (True, False):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                run(keep)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            res[keep].append(ms)
            print(json.dumps({"round": r, "keep_monomials": keep, "lde_ms": round(ms, 3)}), flush=True)
    print(json.dumps({"median_keep_ms": statistics.median(res[True]), "median_drop_ms": statistics.median(res[False])}))


if __name__ == "__main__":
    main()
