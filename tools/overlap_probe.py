#!/usr/bin/env python3
"""Does hashing column chunk k on a second stream while chunk k+1's LDE runs help?

One-GPU commit of a config, three ways, same inputs:
  seq      bj_lde_d (all columns) -> bj_merkle_leaves_d -> nodes, one stream;
  chunked  per column chunk: LDE then partial leaves, one stream;
  overlap  per column chunk: LDE on stream A, partial leaves on stream B after an event
           (the sponge carries its capacity words between chunks, bj_merkle_leaves_partial_d).
Prints ms per commit for each and checks the three caps agree.

usage: python tools/overlap_probe.py [config] [chunk_cols ...]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "era-boojum_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from boojum_amd import commit
    from boojum_amd._lib import call
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
    chunk_list = [int(x) for x in sys.argv[2:]] or [32, 64]
    n_cols, log_n, log_lde, cap = bench.CONFIGS[cfg]
    n, D = 1 << log_n, 1 << log_lde
    nl = n * D
    trace = commit.synthetic_trace(n_cols, log_n)
    ws = commit.CommitWorkspace(n_cols, log_n, log_lde, cap)
    state = torch.empty((nl, 4), dtype=torch.int64, device="cuda")
    sa = torch.cuda.current_stream()
    sb = torch.cuda.Stream()
    # the LDE on a high-priority stream: the dispatcher then places NTT blocks first when a CU
    # frees room (BJ_LEAF_LDS_BYTES caps the leaf blocks per CU so that room exists)
    hp = torch.cuda.Stream(priority=-1)

    def seq():
        st = sa.cuda_stream
        call("bj_lde_d", trace.data_ptr(), n_cols, n, log_n, log_lde, ws.scratch.data_ptr(), ws.lde.data_ptr(), st)
        call("bj_merkle_leaves_d", ws.lde.data_ptr(), n_cols, nl, nl, ws.leaves.data_ptr(), st)
        call("bj_merkle_nodes_d", ws.leaves.data_ptr(), nl, cap, ws.nodes.data_ptr(), st)

    def chunked(cc, two_streams, lde_stream=None):
        k_total = n_cols // cc
        leaf_stream = sb if two_streams else sa
        la = lde_stream or sa
        if lde_stream is not None:
            la.wait_stream(sa)
        evs = []
        for k in range(k_total):
            c0 = k * cc
            call("bj_lde_d", trace[c0].data_ptr(), cc, n, log_n, log_lde, ws.scratch[c0].data_ptr(),
                 ws.lde[c0].data_ptr(), la.cuda_stream)
            e = torch.cuda.Event()
            e.record(la)
            evs.append(e)
        for k in range(k_total):
            c0 = k * cc
            leaf_stream.wait_event(evs[k])
            last = k == k_total - 1
            call("bj_merkle_leaves_partial_d", ws.lde[c0].data_ptr(), cc, nl, nl,
                 None if k == 0 else state.data_ptr(), (ws.leaves if last else state).data_ptr(), 1 if last else 0,
                 leaf_stream.cuda_stream)
        call("bj_merkle_nodes_d", ws.leaves.data_ptr(), nl, cap, ws.nodes.data_ptr(), leaf_stream.cuda_stream)
        if two_streams:
            sa.wait_stream(sb)
        if lde_stream is not None:
            sa.wait_stream(la)

    def timeit(fn, reps=3):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3

    out = {"config": cfg}
    out["seq_ms"] = timeit(seq)
    ref_cap = ws.cap.clone()
    for cc in chunk_list:
        out["chunked%d_ms" % cc] = timeit(lambda: chunked(cc, False))
        assert torch.equal(ws.cap, ref_cap), "chunked cap differs"
        out["overlap%d_ms" % cc] = timeit(lambda: chunked(cc, True))
        assert torch.equal(ws.cap, ref_cap), "overlap cap differs"
        out["overlap%d_hp_ms" % cc] = timeit(lambda: chunked(cc, True, hp))
        assert torch.equal(ws.cap, ref_cap), "overlap (high-priority LDE) cap differs"
    out["leaf_lds_bytes"] = int(os.environ.get("BJ_LEAF_LDS_BYTES", "0"))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
