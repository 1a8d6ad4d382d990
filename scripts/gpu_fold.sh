#!/bin/bash
# Sender-side fold (all-to-all exchange): GPU parity, per-rank compute, gloo rehearsal of the N=4 bench path.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_fold.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_fold.log; exit 1; }
tail -3 gpurun_out/pytest_fold.log
timeout -k 10 300 python tools/shard_compute_probe.py C3 > gpurun_out/probe_fold.log 2>&1 || { echo "probe rc=$?"; tail -20 gpurun_out/probe_fold.log; exit 1; }
tail -1 gpurun_out/probe_fold.log
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 4 --steps 2 --warmup 1 --config C2 --dist-backend gloo > gpurun_out/rehearse4.log 2>&1 || { echo "rehearse rc=$?"; tail -30 gpurun_out/rehearse4.log; exit 1; }
tail -1 gpurun_out/rehearse4.log
