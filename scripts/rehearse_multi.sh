#!/bin/bash
# N>1 bench path rehearsal on one GPU (gloo staging, ranks share the card): not a benchmark.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --config C2 --dist-backend gloo > gpurun_out/rehearse2.log 2>&1 || { echo "rehearse rc=$?"; tail -30 gpurun_out/rehearse2.log; exit 1; }
tail -2 gpurun_out/rehearse2.log
