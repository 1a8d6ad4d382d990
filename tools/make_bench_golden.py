#!/usr/bin/env python3
"""Golden caps of the bench configs (tests/golden/bench_caps.json), from the CPU oracle.

bench.py's verify step compares every rank's cap of the synthetic trace (SURVEY 8(d):
splitmix64(42 + c n + r) mod p) with these.  Each entry is the cap of the oracle's commit
(oracle/boojum_oracle.c, the restatement of prover.rs:313-353 the tests check the GPU against),
so a verified bench line is bit-exact against the reference's algorithm end to end.  Test
infrastructure: only the bench's verify step and the tests read the file.

C3 needs ~45 GiB of host memory (trace + LDE) and ~10^9 oracle permutations: run it where
that fits (the GPU box host), e.g.
    python tools/make_bench_golden.py C3 --threads 16
`--chunk-cols K` (Poseidon2 only) commits K columns at a time instead: the LDE of a column
chunk, then the leaf sponges carried over it (bjo_poseidon2_leaves_partial), so C4 (2^23 x 256,
LDE x8: 128 GiB of LDE) needs ~10 GiB at K = 8.  Same cap: the sponge is sequential over the
row's elements and a chunk boundary on a multiple of 8 columns is a rate boundary.

usage: python tools/make_bench_golden.py CONFIG[/HASHER] ... [--threads T]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import oracle as O
    from bench import CONFIGS, GOLDEN_CAPS
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="+")
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--out", default=GOLDEN_CAPS)
    ap.add_argument("--chunk-cols", type=int, default=0)
    args = ap.parse_args()
    try:
        data = json.load(open(args.out))
    except OSError:
        data = {"note": "caps of the bench configs' synthetic traces from the CPU oracle (tools/make_bench_golden.py)",
                "caps": {}}
    for spec in args.configs:
        cfg, _, hasher = spec.partition("/")
        hasher = hasher or "poseidon2"
        n_cols, log_n, log_lde, cap = CONFIGS[cfg]
        t0 = time.time()
        if args.chunk_cols:
            assert hasher == "poseidon2" and args.chunk_cols % 8 == 0
            state = None
            for c0 in range(0, n_cols, args.chunk_cols):
                k = min(args.chunk_cols, n_cols - c0)
                _, lde = O.lde(O.synthetic_trace(k, log_n, col_offset=c0), log_lde, threads=args.threads)
                state = O.poseidon2_leaves_partial(lde.reshape(k, -1), state, c0 + k == n_cols, threads=args.threads)
                del lde
                print("  %s columns %d..%d  %.0f s" % (cfg, c0, c0 + k, time.time() - t0), flush=True)
            cap_v = O.merkle_nodes(state, cap, threads=args.threads)[1]
            how = "oracle LDE + leaf sponges in %d-column chunks" % args.chunk_cols
        elif hasher == "poseidon2":
            how = "oracle lde_commit"
            ref = O.lde_commit(O.synthetic_trace(n_cols, log_n), log_lde, cap, threads=args.threads, in_place=True)
            cap_v = ref["cap"]
        else:
            how = "oracle lde_commit"
            _, lde = O.lde(O.synthetic_trace(n_cols, log_n), log_lde, threads=args.threads)
            cap_v = O.merkle_construct(lde.reshape(n_cols, -1), cap, threads=args.threads, hasher=hasher)[3]
        data["caps"]["%s/%s" % (cfg, hasher)] = {
            "cap": [["%016x" % int(x) for x in row] for row in np.asarray(cap_v, dtype=np.uint64)],
            "source": "%s, %d threads, %.0f s" % (how, args.threads, time.time() - t0)}
        print(spec, "done in %.0f s" % (time.time() - t0), flush=True)
        with open(args.out, "w") as f:
            json.dump(data, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
