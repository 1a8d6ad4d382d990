#!/bin/bash
# First GPU pass: VALU microbench, GPU parity tests, short benches.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/microbench_valu > gpurun_out/micro.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || exit $?
echo done
