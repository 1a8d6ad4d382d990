#!/usr/bin/env python3
"""How expensive is pinning caller memory (hipHostRegister) against the pageable copy path?
Times register / D2H into registered memory / unregister for a few sizes, and a pageable D2H.
A sizing probe for bj_lde_commit_h's host pipeline, not product code."""
import ctypes
import time

import numpy as np
import torch


def main():
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    torch.cuda.init()
    for gib in (0.5, 2):
        nbytes = int(gib * (1 << 30))
        host = np.empty(nbytes // 8, dtype=np.uint64)
        host[::512] = 1  # touch the pages
        dev = torch.empty(nbytes // 8, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rc = hip.hipMemcpy(host.ctypes.data, dev.data_ptr(), nbytes, 2)
        t1 = time.perf_counter()
        rc |= hip.hipHostRegister(host.ctypes.data, nbytes, 0)
        t2 = time.perf_counter()
        rc |= hip.hipMemcpy(host.ctypes.data, dev.data_ptr(), nbytes, 2)
        t3 = time.perf_counter()
        rc |= hip.hipMemcpy(dev.data_ptr(), host.ctypes.data, nbytes, 1)
        t4 = time.perf_counter()
        rc |= hip.hipHostUnregister(host.ctypes.data)
        t5 = time.perf_counter()
        print({"GiB": gib, "rc": rc, "pageable_d2h_GBs": round(nbytes / (t1 - t0) / 1e9, 1),
               "register_ms": round((t2 - t1) * 1e3, 1), "pinned_d2h_GBs": round(nbytes / (t3 - t2) / 1e9, 1),
               "pinned_h2d_GBs": round(nbytes / (t4 - t3) / 1e9, 1), "unregister_ms": round((t5 - t4) * 1e3, 1)})


if __name__ == "__main__":
    main()
