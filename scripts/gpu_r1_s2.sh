#!/bin/bash
# Session-2 first GPU pass: ISA rate microbench, GPU tests, C3 bench, rocprof stats.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/microbench_isa > gpurun_out/isa.log 2>&1 || { echo "isa rc=$?"; exit 1; }
timeout -k 10 120 ./tools/microbench_valu > gpurun_out/valu.log 2>&1 || { echo "valu rc=$?"; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_s2.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_s2.log; exit 1; }
tail -3 gpurun_out/pytest_s2.log
timeout -k 10 300 python -u bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_s2.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_s2.log; exit 1; }
tail -1 gpurun_out/bench_s2.log
echo done
