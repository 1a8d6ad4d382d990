#!/usr/bin/env python3
"""PCIe sizing probe for the host-buffer commit (bj_lde_commit_h): pinned vs pageable copies,
one direction and both at once, and the host's multi-threaded memcpy rate.  Not product code.
usage: python tools/duplex_probe.py"""
import json
import threading
import time

import numpy as np
import torch


def timed(fn, reps=3):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


def main():
    nb = 1 << 30
    n = nb // 8
    dev_a = torch.empty(n, dtype=torch.int64, device="cuda")
    dev_b = torch.empty(n, dtype=torch.int64, device="cuda")
    pin_a = torch.empty(n, dtype=torch.int64, pin_memory=True)
    pin_b = torch.empty(n, dtype=torch.int64, pin_memory=True)
    pag_a = torch.from_numpy(np.ones(n, dtype=np.int64))
    pag_b = torch.from_numpy(np.ones(n, dtype=np.int64))
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    out = {}

    def both(h_in, h_out):
        with torch.cuda.stream(s1):
            dev_a.copy_(h_in, non_blocking=True)
        with torch.cuda.stream(s2):
            h_out.copy_(dev_b, non_blocking=True)
        s1.synchronize()
        s2.synchronize()

    out["pinned_h2d_GBs"] = nb / timed(lambda: dev_a.copy_(pin_a, non_blocking=True)) / 1e9
    out["pinned_d2h_GBs"] = nb / timed(lambda: pin_b.copy_(dev_b, non_blocking=True)) / 1e9
    out["pinned_duplex_GBs_each"] = nb / timed(lambda: both(pin_a, pin_b)) / 1e9
    out["pageable_h2d_GBs"] = nb / timed(lambda: dev_a.copy_(pag_a)) / 1e9
    out["pageable_d2h_GBs"] = nb / timed(lambda: pag_b.copy_(dev_b)) / 1e9
    out["pageable_duplex_GBs_each"] = nb / timed(lambda: both(pag_a, pag_b)) / 1e9
    src = np.ones(n, dtype=np.uint64)
    dst = np.empty(n, dtype=np.uint64)
    for th in (1, 4, 8, 16):
        parts = np.array_split(np.arange(n), th)

        def work(lo, hi):
            np.copyto(dst[lo:hi], src[lo:hi])

        def run():
            ts = [threading.Thread(target=work, args=(p[0], p[-1] + 1)) for p in parts]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
        out["host_memcpy_GBs_%dthreads" % th] = nb / timed(run) / 1e9
    print(json.dumps({k: round(v, 1) for k, v in out.items()}))


if __name__ == "__main__":
    main()
