#!/bin/bash
# The plain-C caller at 1..16 seam threads, then the whole GPU suite without -x.
cd "$GRAFT_REPO_ROOT"
for t in 1 1 1 8 8 8 16 16; do
    timeout -k 5 60 ./tests/c/c_caller 16 32 1 16 $t > gpurun_out/cc_$t.log 2>&1
    echo "threads=$t rc=$?"
    tail -n 2 gpurun_out/cc_$t.log
done
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/mad_tests2.log 2>&1
echo "pytest rc=$?"
tail -n 15 gpurun_out/mad_tests2.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/mad_bench.log 2>&1
echo "bench rc=$?"
tail -n 1 gpurun_out/mad_bench.log
