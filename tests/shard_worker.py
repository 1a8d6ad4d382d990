"""One rank of a multi-process sharded commit (spawned by test_sharded_*.py).

Writes rank<P>.npz with its lde slice, leaves, nodes and cap into `outdir`."""
import os
import sys


def run(rank, world, port, cfg, outdir, device, paths):
    for p in paths:
        if p not in sys.path:
            sys.path.insert(0, p)
    import numpy as np
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from boojum_amd.sharded import ShardedWorkspace, sharded_witness_commit
        n_cols, log_n, log_lde, cap = cfg[:4]
        extra = {"max_chunk_cols": 8 * cfg[4]} if len(cfg) > 4 and cfg[4] else {}
        if len(cfg) > 5 and cfg[5] is not None:
            extra["fold_exchange"] = cfg[5]
        hasher = cfg[6] if len(cfg) > 6 else "poseidon2"
        if device == "cpu":
            from shard_cpu_ops import CpuShardOps
            ops, dev = CpuShardOps(hasher), "cpu"
        else:
            torch.cuda.set_device(0)
            ops, dev = None, "cuda:0"
            extra["hasher"] = hasher
        ws = ShardedWorkspace(n_cols, log_n, log_lde, cap, rank, world, device=dev, ops=ops, **extra)
        tr = ws.synthetic_trace_shard()
        sharded_witness_commit(tr, ws)
        if dev != "cpu":
            torch.cuda.synchronize()
        u = lambda t: t.cpu().numpy().view(np.uint64)  # noqa: E731
        from boojum_amd.sharded import sharded_query
        nl = ws.m * world
        qidx = sorted({0, nl - 1, nl // 3, ws.m, (5 * nl) // 7})
        qs = [sharded_query(ws, i) for i in qidx]
        np.savez(os.path.join(outdir, "rank%d.npz" % rank), lde=u(ws.lde), leaves=u(ws.leaves), nodes=u(ws.nodes),
                 cap=u(ws.cap), qidx=np.array(qidx), q_elems=np.stack([u(q[0]) for q in qs]),
                 q_leaf=np.stack([u(q[1]) for q in qs]), q_path=np.stack([u(q[2]) for q in qs]))
    finally:
        dist.destroy_process_group()
