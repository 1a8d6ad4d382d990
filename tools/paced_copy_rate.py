#!/usr/bin/env python3
"""Rates the RCCL-shaped stand-in (tools/paced_copy.hip) reaches on one GPU, unpaced and paced."""
# measure the stand-in's unpaced and paced rates on one GPU
import ctypes, torch, os, time
lib = ctypes.CDLL(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tools", "libpaced_copy.so"))
lib.paced_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, ctypes.c_double, ctypes.c_void_p]
ring = 512 << 20
a = torch.empty(ring // 8, dtype=torch.int64, device="cuda"); b = torch.empty_like(a)
st = torch.cuda.current_stream()
tot = 4 << 30
for ch in (8, 16, 32, 64):
    for gbps in (0.0, 64.0, 200.0, 450.0):
        lib.paced_copy(a.data_ptr(), b.data_ptr(), ring, 1 << 28, ch, gbps, st.cuda_stream); torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); rc = lib.paced_copy(a.data_ptr(), b.data_ptr(), ring, tot, ch, gbps, st.cuda_stream); e.record(); torch.cuda.synchronize()
        print("channels %2d target %5.0f GB/s -> %6.1f GB/s" % (ch, gbps, tot / (s.elapsed_time(e) * 1e-3) / 1e9), flush=True)
