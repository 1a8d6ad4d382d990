#!/bin/bash
# Per-rank compute of the sharded commit (G = 1..8, exchange stubbed) and the bench's N>1
# path rehearsed through gloo with 4 ranks on one card (C2).
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/shard_compute_probe.py C3 > gpurun_out/probe_r1s.log 2>&1 || { echo "probe rc=$?"; tail -20 gpurun_out/probe_r1s.log; exit 1; }
tail -n 1 gpurun_out/probe_r1s.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29531 \
    bench.py --gpus 4 --steps 2 --warmup 1 --config C2 --dist-backend gloo > gpurun_out/rehearse4_r1s.log 2>&1 || { echo "rehearse rc=$?"; tail -20 gpurun_out/rehearse4_r1s.log; exit 1; }
tail -n 1 gpurun_out/rehearse4_r1s.log
