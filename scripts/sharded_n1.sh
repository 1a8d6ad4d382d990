#!/bin/bash
# The sharded (column-pipelined) runner at N=1 vs the single-GPU runner, C3.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --sharded > gpurun_out/sharded_n1.log 2>&1 || { echo "sharded rc=$?"; tail -20 gpurun_out/sharded_n1.log; exit 1; }
tail -1 gpurun_out/sharded_n1.log
timeout -k 10 600 python -u bench.py --config C4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/c4_n1.log 2>&1 || { echo "c4 rc=$?"; tail -20 gpurun_out/c4_n1.log; exit 1; }
tail -1 gpurun_out/c4_n1.log
