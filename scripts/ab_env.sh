#!/bin/bash
# A/B of an environment switch on the C3 bench: parity tests first, then the bench with each
# setting, then a kernel trace of the default.  usage: bash scripts/ab_env.sh TAG VAR VALUE_B [tests]
set -u
TAG=$1; VAR=$2; VB=$3; TESTS=${4:-"tests/test_gpu_parity.py tests/test_gpu_fullsize.py"}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_${TAG}.log; exit 1; }
tail -2 gpurun_out/pytest_${TAG}.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_${TAG}_A.log 2>&1 || { echo "bench A failed"; tail -20 gpurun_out/bench_${TAG}_A.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_A.log | cut -c1-420
env $VAR=$VB timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_${TAG}_B.log 2>&1 || { echo "bench B failed"; tail -20 gpurun_out/bench_${TAG}_B.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_B.log | cut -c1-420
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1 || { echo "prof failed"; exit 1; }
head -14 gpurun_out/prof_${TAG}/run_kernel_stats.csv | cut -c1-160
echo done
