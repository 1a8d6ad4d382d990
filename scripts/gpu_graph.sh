#!/bin/bash
# HIP-graph commit replay: parity test, then eager vs graph benches at C5 and C3.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_oracles.py -x -q --timeout 120 --timeout-method thread -k graph > gpurun_out/graph_test.log 2>&1 || { echo "test failed"; tail -30 gpurun_out/graph_test.log; exit 1; }
tail -1 gpurun_out/graph_test.log
for args in "--config C5" "--config C5 --graph" "--config C5 --hasher blake2s" "--config C5 --hasher blake2s --graph" "--config C3 --graph"; do
  timeout -k 10 300 python -u bench.py $args --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/graph_bench.log 2>&1 || { echo "bench $args failed"; tail -20 gpurun_out/graph_bench.log; exit 1; }
  tail -1 gpurun_out/graph_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$args', round(d['ms_per_step'],4), d['phase_ms'])"
done
