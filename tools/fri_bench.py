#!/usr/bin/env python3
"""Measurement of SURVEY 8(f) row 3 (FRI) at the C3 codeword size: one fold by 2
(bj_fri_fold_d, fold_multiple fri/mod.rs:362-474) and the FRI oracle tree's leaf hashing
(bj_merkle_leaves_chunked_d, construct_by_chunking merkle_tree.rs:176-306), timed with HIP events
on the stream they run on, each against its roofline.

* fold: algorithmic bytes per launch = N*8*2 (c0, c1 read) + N/2*8 (roots) + N/2*8*2 (outputs),
  N = codeword length; bound HBM (8 TB/s).
* chunked leaves: 2 columns (c0, c1) x E elements per leaf = ceil(2E/8) Poseidon2 permutations
  per leaf; bound VALU issue (the permutation's issue slots, boojum_amd/valu_census.json).

usage: python tools/fri_bench.py [log_n=24] [log_e=3]   (prints one JSON line)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "era-boojum_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0
VALU_PEAK_TSLOTS = 78.6432


def timed(torch, fn, reps=20):
    st = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    import torch
    from boojum_amd import fri
    from boojum_amd._lib import call
    from boojum_amd.field import stream_of
    log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    log_e = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    n = 1 << log_n
    c = torch.empty((2, n), dtype=torch.int64, device="cuda")
    call("bj_fill_synthetic_d", c.data_ptr(), 2, n, log_n, 7, 0, stream_of(c))
    roots = fri.precompute_roots(n)
    ch = (123456789, 987654321)
    t_fold = timed(torch, lambda: fri.fold(c[0], c[1], roots, 3, ch))
    fold_bytes = n * 16 + (n // 2) * 8 + (n // 2) * 16
    e = 1 << log_e
    nl = n // e
    out = torch.empty((nl, 4), dtype=torch.int64, device="cuda")
    t_leaves = timed(torch, lambda: call("bj_merkle_leaves_chunked_d", c.data_ptr(), 2, n, nl, e, out.data_ptr(),
                                         stream_of(out)))
    census = json.load(open(os.path.join(ROOT, "era-boojum_amd", "boojum_amd", "valu_census.json")))
    import bench
    slots = bench.leaf_slots_per_perm(census, 2 * e)
    perms = nl * ((2 * e + 7) // 8)
    line = {
        "codeword": "GoldilocksExt2 x 2^%d (C3 FRI base oracle size)" % log_n,
        "fold": {"ms": t_fold * 1e3, "bound": "hbm", "achieved": fold_bytes / t_fold / 1e9, "peak": HBM_PEAK_GBS,
                 "unit": "GB/s", "frac": fold_bytes / t_fold / 1e9 / HBM_PEAK_GBS, "alg_bytes_per_launch": fold_bytes},
        "chunked_leaves": {"elems_per_leaf": e, "leaves": nl, "ms": t_leaves * 1e3, "bound": "valu",
                           "achieved": perms * slots / t_leaves / 1e12, "peak": VALU_PEAK_TSLOTS, "unit": "Tslot/s",
                           "frac": perms * slots / t_leaves / 1e12 / VALU_PEAK_TSLOTS, "perms_per_launch": perms},
    }
    print(json.dumps(line))


if __name__ == "__main__":
    main()
