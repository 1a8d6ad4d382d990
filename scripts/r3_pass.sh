#!/bin/bash
# Round-3 development pass: every GPU test on the current library, then same-box A/Bs of the C3
# bench: the library against libboojum_mi355x.so.old (a previous build, swapped in and out) and
# the three-pass LDE against BJ_LDE_PASSES=2; then the LDE ablation tool.
# usage: bash scripts/r3_pass.sh TAG [notests]
set -u
TAG=${1:-r3}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
O=gpurun_out/$TAG
L=era-boojum_amd/boojum_amd/libboojum_mi355x.so
if [ "${2:-}" = "quick" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_lde3.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "lde or fft or transforms or commit" > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest.log | head; tail -20 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
elif [ "${2:-}" != "notests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest.log | head; tail -20 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
cp $L $L.new
B="python3 -u bench.py --config C3 --steps 8 --warmup 2 --no-cpu-baseline --no-native-base"
summ() { python3 -c "import json,sys;l=[x for x in open(sys.argv[1]) if x.startswith('{')][-1];d=json.loads(l);print(round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['phase_ms'].items()},d['verified'])" $1; }
for V in old new old new; do
  cp $L.$V $L
  timeout -k 10 200 $B > $O/bench_$V.log 2>&1 || { echo "bench $V failed"; tail -5 $O/bench_$V.log; cp $L.new $L; exit 1; }
  echo "lib $V: $(summ $O/bench_$V.log)"
done
cp $L.new $L
for i in 1 2; do
  BJ_LDE_PASSES=2 timeout -k 10 200 $B > $O/bench_2pass_$i.log 2>&1 || { echo "bench 2pass failed"; exit 1; }
  echo "2-pass LDE: $(summ $O/bench_2pass_$i.log)"
done
if [ -x tools/lde3_ablation ]; then
  timeout -k 10 120 ./tools/lde3_ablation > $O/lde3_ablation.log 2>&1 || { echo "ablation failed"; exit 1; }
  cat $O/lde3_ablation.log
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
python3 -c "
import csv,sys
for r in csv.DictReader(open('$O/trace/run_kernel_stats.csv')):
    print('%-70s %5s %9.3f ms' % (r['Name'][:70].replace('void bj::(anonymous namespace)::',''), r['Calls'], float(r['AverageNs'])/1e6))
" | head -8
echo done
