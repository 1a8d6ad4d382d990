#!/bin/bash
# Native collective commit: GPU parity (in-process ranks + RCCL at world 1), then the C3 bench
# through bj_sharded_commit_d at N = 1 beside the default path.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_native_sharded.py -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_native.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_native.log; exit 1; }
tail -3 gpurun_out/pytest_native.log
timeout -k 10 300 python -u bench.py --native --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_native.log 2>&1 || { echo "bench native rc=$?"; tail -20 gpurun_out/bench_native.log; exit 1; }
tail -1 gpurun_out/bench_native.log | cut -c1-600
