#!/bin/bash
# Standard GPU pass: GPU tests, the C3 bench (N = 1), and optionally the N = 4 gloo rehearsal
# of the native collective (C2) and a rocprof kernel trace.  Each GPU step has its own time
# limit; the first failure ends the script.
# usage: bash scripts/gpu_check.sh TAG [bench steps] [multi] [prof]
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
if [ "${3:-}" = "multi" ]; then
  timeout -k 10 300 python -u bench.py --gpus 4 --dist-backend gloo --config C2 --steps 2 --warmup 1 > gpurun_out/bench_gloo4_${TAG}.log 2>&1 || { echo "gloo x4 bench failed"; tail -20 gpurun_out/bench_gloo4_${TAG}.log; exit 1; }
  tail -1 gpurun_out/bench_gloo4_${TAG}.log
fi
if [ "${4:-}" = "prof" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1 || { echo "prof failed"; exit 1; }
  head -12 gpurun_out/prof_${TAG}/run_kernel_stats.csv | cut -c1-200
fi
echo done
