#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/microbench_isa > gpurun_out/isa.log 2>&1 || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1a -o run -- python3 bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r1a.log 2>&1 || exit $?
echo done
