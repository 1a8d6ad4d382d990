#!/bin/bash
# Standard GPU pass: GPU tests, then the C3 bench (and optionally a rocprof kernel trace).
# usage: bash scripts/gpu_check.sh TAG [bench steps] [prof]
set -u
TAG=${1:-run}
STEPS=${2:-3}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAIL|Error|error" gpurun_out/pytest_${TAG}.log | head -20; tail -30 gpurun_out/pytest_${TAG}.log; exit 1; }
tail -3 gpurun_out/pytest_${TAG}.log
timeout -k 10 300 python -u bench.py --config C3 --steps $STEPS --warmup 1 --no-cpu-baseline > gpurun_out/bench_${TAG}.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_${TAG}.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}.log
if [ "${3:-}" = "prof" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1 || { echo "prof failed"; exit 1; }
  head -12 gpurun_out/prof_${TAG}/run_kernel_stats.csv | cut -c1-200
fi
echo done
