#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-buffer boundary (bj_lde_commit_h): the trace copied in from
host memory, every output (LDE, leaves, nodes, cap) copied back.  Reported in DESIGN.md beside
the device-resident bench value; never the bench's `value`.

usage: python tools/host_resident.py [log_n] [n_cols] [log_lde] [pinned]
"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "era-boojum_amd"))


def main():
    from boojum_amd._lib import call
    log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    c = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    log_d = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    cap = 16
    n, nl = 1 << log_n, 1 << (log_n + log_d)
    p = ctypes.POINTER(ctypes.c_uint64)
    tr = np.random.default_rng(1).integers(0, 2**63, size=(c, n), dtype=np.uint64)
    lde = np.empty((c, nl), dtype=np.uint64)
    leaves = np.empty((nl, 4), dtype=np.uint64)
    nodes = np.empty((nl - cap, 4), dtype=np.uint64)
    capo = np.empty((cap, 4), dtype=np.uint64)
    args = (tr.ctypes.data_as(p), c, log_n, log_d, log_d, cap, lde.ctypes.data_as(p), leaves.ctypes.data_as(p),
            nodes.ctypes.data_as(p), capo.ctypes.data_as(p))
    pinned = len(sys.argv) > 4 and sys.argv[4] == "pinned"
    if pinned:
        # callers that reuse their buffers can page-lock them once (hipHostRegister), so the
        # copies DMA straight to / from them instead of pinning on the fly per call
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
        for a in (tr, lde, leaves, nodes):
            assert hip.hipHostRegister(a.ctypes.data, a.nbytes, 0) == 0
    call("bj_lde_commit_h", *args)   # warm-up (tables, allocator)
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        call("bj_lde_commit_h", *args)
    dt = (time.perf_counter() - t0) / reps
    moved = 8 * c * n + 8 * c * nl + 32 * nl + 32 * (nl - cap)
    print('{"config": "2^%d x %d, LDE x%d", "host_buffers": "%s", "ms_per_commit": %.1f, "trace_elems_per_s": %.4g, '
          '"host_bytes_moved": %d}' % (log_n, c, 1 << log_d, "registered" if pinned else "pageable", dt * 1e3,
                                        c * n / dt, moved))


if __name__ == "__main__":
    main()
