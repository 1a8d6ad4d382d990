"""One rank of a multi-process sharded commit (spawned by sharded_check.run_and_check).

device "cpu": the CPU model of the native schedule (sharded_model.py) with the oracle's steps;
device "cuda": the product, bj_sharded_commit_d, over the torch.distributed (gloo) group through
the callback transport, all ranks sharing the one GPU.  Writes rank<P>.npz with its LDE blocks,
leaves, nodes, cap and a few openings into `outdir`.

cfg = (n_cols, log_n, log_lde, cap[, max_chunk_units[, fold_exchange[, hasher[, log_k]]]])."""
import os
import sys


def run(rank, world, cfg, outdir, device, paths):
    for p in paths:
        if p not in sys.path:
            sys.path.insert(0, p)
    import numpy as np
    import torch
    import torch.distributed as dist

    # rendezvous through a file in the test's own directory: no TCP port to collide with
    dist.init_process_group("gloo", init_method="file://" + os.path.join(outdir, "rendezvous"), rank=rank,
                            world_size=world)
    try:
        n_cols, log_n, log_lde, cap = cfg[:4]
        hasher = cfg[6] if len(cfg) > 6 and cfg[6] else "poseidon2"
        log_k = cfg[7] if len(cfg) > 7 and cfg[7] is not None else log_lde
        nl = (1 << log_n) << log_k
        m = nl // world
        qidx = sorted({0, nl - 1, nl // 3, m, (5 * nl) // 7})
        u = lambda t: t.cpu().numpy().view(np.uint64)  # noqa: E731
        if device == "cpu":
            import sharded_model as SM
            from shard_cpu_ops import CpuShardOps
            extra = {"max_chunk_cols": 8 * cfg[4]} if len(cfg) > 4 and cfg[4] else {}
            if len(cfg) > 5 and cfg[5] is not None:
                extra["fold_exchange"] = cfg[5]
            ws = SM.ShardModel(n_cols, log_n, log_lde, cap, rank, world, CpuShardOps(hasher), log_k=log_k,
                               hasher=hasher, **extra)
            SM.commit(ws.synthetic_trace_shard(), ws)
            qs = [SM.query(ws, i) for i in qidx]
            out = dict(lde=u(ws.lde), leaves=u(ws.leaves), nodes=u(ws.nodes), cap=u(ws.cap))
            qs = [tuple(u(t) for t in q) for q in qs]
        else:
            from boojum_amd._lib import call
            from boojum_amd.field import stream_of
            from boojum_amd.sharded import NativeComm, native_columns, native_sharded_commit, native_sharded_query
            torch.cuda.set_device(0)
            comm = NativeComm.torch_dist()
            try:
                cols = native_columns(n_cols, world, rank, hasher)
                n = 1 << log_n
                tr = torch.empty((len(cols), n), dtype=torch.int64, device="cuda")
                for j, c in enumerate(cols):
                    call("bj_fill_synthetic_d", tr[j].data_ptr(), 1, n, log_n, 42, c, stream_of(tr))
                r = native_sharded_commit(comm, tr, n_cols, log_n, log_lde, cap, hasher, log_commit_cosets=log_k)
                torch.cuda.synchronize()
                qs = [native_sharded_query(comm, r, n_cols, log_n, log_lde, cap, i, hasher, log_commit_cosets=log_k)
                      for i in qidx]
                out = dict(lde=u(r.lde), leaves=u(r.leaves), nodes=u(r.nodes), cap=u(r.cap))
            finally:
                comm.close()
        np.savez(os.path.join(outdir, "rank%d.npz" % rank), qidx=np.array(qidx),
                 q_elems=np.stack([q[0] for q in qs]), q_leaf=np.stack([q[1] for q in qs]),
                 q_path=np.stack([q[2] for q in qs]), **out)
    finally:
        dist.destroy_process_group()
