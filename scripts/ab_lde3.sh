#!/bin/bash
# Three-pass LDE check: its parity tests first, then every GPU test, then a same-box A/B of the
# C3 bench (three passes vs BJ_LDE_PASSES=2, alternated) and a kernel trace of each.
# usage: bash scripts/ab_lde3.sh TAG [full]
set -u
TAG=${1:-lde3}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
O=gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_lde3.py -x -v --timeout 120 --timeout-method thread > $O/pytest_lde3.log 2>&1 || { echo "lde3 tests failed"; grep -E "FAIL|Error|assert" $O/pytest_lde3.log | head -20; tail -30 $O/pytest_lde3.log; exit 1; }
tail -1 $O/pytest_lde3.log
if [ "${2:-}" = "full" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest.log | head; tail -20 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
B="python3 -u bench.py --config C3 --steps 10 --warmup 2 --no-cpu-baseline --no-native-base"
for i in 1 2; do
  timeout -k 10 300 $B > $O/bench3_$i.log 2>&1 || { echo "bench3 failed"; tail -20 $O/bench3_$i.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"lde": [0-9.]*\|"verified": [a-z]*' $O/bench3_$i.log | tr '\n' ' '; echo " <- 3-pass"
  BJ_LDE_PASSES=2 timeout -k 10 300 $B > $O/bench2_$i.log 2>&1 || { echo "bench2 failed"; tail -20 $O/bench2_$i.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"lde": [0-9.]*\|"verified": [a-z]*' $O/bench2_$i.log | tr '\n' ' '; echo " <- 2-pass"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace3 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-native-base > $O/trace3.log 2>&1 || { echo "trace failed"; exit 1; }
head -8 $O/trace3/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-160
echo done
