#!/bin/bash
# GPU suite, then the C5 / C2 / C3 benches (small-size CT heads, node-tail threshold).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_small.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAIL|Error" gpurun_out/pytest_small.log | head -20; tail -30 gpurun_out/pytest_small.log; exit 1; }
tail -2 gpurun_out/pytest_small.log
for c in C5 C2 C3; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_small_$c.log 2>&1 || { echo "bench $c failed"; tail -20 gpurun_out/bench_small_$c.log; exit 1; }
  tail -1 gpurun_out/bench_small_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'], round(d['ms_per_step'],3), d['phase_ms'])"
done
timeout -k 10 300 python -u bench.py --config C5 --hasher blake2s --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_small_C5b.log 2>&1 && tail -1 gpurun_out/bench_small_C5b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'], round(d['ms_per_step'],3), d['phase_ms'])"
