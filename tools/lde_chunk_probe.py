"""Column-chunked LDE probe: does running the three LDE passes over a few columns at a time (so a
chunk's intermediates, c x D x 32 MiB at C3, can stay in the 256 MB Infinity Cache between the
passes) beat one call over all 256 columns?  Same C3 workload, same outputs (checked), HIP events
on the work stream; eager launches and the same launches replayed from a captured graph.
Prints one JSON line per variant and repetition, then the medians."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "era-boojum_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", default="1,2,4,8,32")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--log-n", type=int, default=22)
    ap.add_argument("--cols", type=int, default=256)
    ap.add_argument("--log-d", type=int, default=2)
    ap.add_argument("--graph", type=int, default=1)
    a = ap.parse_args()
    import torch
    from boojum_amd import commit
    from boojum_amd._lib import call
    C, log_n, log_d = a.cols, a.log_n, a.log_d
    n, D = 1 << log_n, 1 << a.log_d
    trace = commit.synthetic_trace(C, log_n)
    scratch = torch.empty((C, n), dtype=torch.int64, device="cuda")
    lde = torch.empty((C, D, n), dtype=torch.int64, device="cuda")
    st = torch.cuda.Stream()
    torch.cuda.synchronize()  # the trace is made on the default stream

    def run(c):
        s = st.cuda_stream
        if c >= C:
            call("bj_lde_ex_d", trace.data_ptr(), C, n, log_n, log_d, scratch.data_ptr(), lde.data_ptr(), 0, s)
            return
        for j in range(0, C, c):
            call("bj_lde_ex_d", trace[j].data_ptr(), c, n, log_n, log_d, scratch.data_ptr(), lde[j].data_ptr(), 0, s)

    def digest():
        v = lde.view(-1)[:: 4099]
        return int(torch.sum(v).item()), int(torch.sum(v * 3 + 1).item())

    chunks = [int(x) for x in a.chunks.split(",")] + [C]
    with torch.cuda.stream(st):
        run(C)
    torch.cuda.synchronize()
    ref = digest()
    graphs = {}
    for c in chunks:
        with torch.cuda.stream(st):
            lde.zero_()  # on the work stream: ordered before the run
            run(c)
        torch.cuda.synchronize()
        dg = digest()
        print(json.dumps({"chunk_cols": c, "digest": dg, "ref": ref, "match": dg == ref}), flush=True)
        if a.graph and c < C:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                run(c)
            torch.cuda.synchronize()
            lde.zero_()
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            dg = digest()
            print(json.dumps({"chunk_cols": c, "mode": "graph", "digest": dg, "match": dg == ref}), flush=True)
            graphs[c] = g
    res = {}
    for r in range(a.rounds):
        for c in chunks:
            for mode in (("eager", "graph") if c in graphs else ("eager",)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                with torch.cuda.stream(st):
                    e0.record(st)
                    for _ in range(a.reps):
                        if mode == "graph":
                            graphs[c].replay()
                        else:
                            run(c)
                    e1.record(st)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.reps
                res.setdefault((c, mode), []).append(ms)
                print(json.dumps({"round": r, "chunk_cols": c, "mode": mode, "lde_ms": round(ms, 3)}), flush=True)
    print(json.dumps({"%d_%s" % k: round(statistics.median(v), 3) for k, v in res.items()}))


if __name__ == "__main__":
    main()
