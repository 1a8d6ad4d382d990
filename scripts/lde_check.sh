# usage: bash scripts/lde_check.sh TAG  -- LDE parity tests, a bench line and a kernel-trace summary
set -u
TAG=$1
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
O=gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests/test_gpu_lde3.py tests/test_gpu_parity.py tests/test_gpu_native_sharded.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-native-base > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
python3 -c "
import json;l=[json.loads(x) for x in open('$O/bench.log') if x.startswith('{')][-1]
print({k:l.get(k) for k in ('ms_per_step','verified','phase_ms')})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-native-base > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('$O/trace/run_kernel_stats.csv')):
    print('%-60s %6s %10.3f' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e6))" | head -12
