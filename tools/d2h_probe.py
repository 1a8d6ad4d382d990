#!/usr/bin/env python3
"""Device-to-host copy rate by piece size and stream count (sizing bj_lde_commit_h's copy-out).
Not product code.  usage: python tools/d2h_probe.py"""
import json
import time

import torch


def rate(nbytes, fn, reps=5):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return round(nbytes / best / 1e9, 1)


def main():
    total = 1 << 30
    n = total // 8
    dev = torch.empty(n, dtype=torch.int64, device="cuda")
    pin = torch.empty(n, dtype=torch.int64, pin_memory=True)
    streams = [torch.cuda.Stream() for _ in range(4)]
    out = {}
    for piece_mib in (16, 64, 256, 1024):
        k = (piece_mib << 20) // 8

        def pieces(ns):
            for i in range(0, n, k):
                s = streams[(i // k) % ns]
                with torch.cuda.stream(s):
                    pin[i:i + k].copy_(dev[i:i + k], non_blocking=True)
            for s in streams[:ns]:
                s.synchronize()
        for ns in (1, 2, 4):
            out["d2h_%dMiB_%dstreams_GBs" % (piece_mib, ns)] = rate(total, lambda: pieces(ns))
        out["h2d_%dMiB_1stream_GBs" % piece_mib] = rate(total, lambda: [dev[i:i + k].copy_(pin[i:i + k], non_blocking=True)
                                                                         for i in range(0, n, k)])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
