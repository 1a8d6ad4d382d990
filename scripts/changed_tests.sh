# The GPU tests of the collective, the C caller, the LDE and the full-size caps, then a bench line
# with the native same-path base.  usage: bash scripts/changed_tests.sh TAG
set -u
TAG=${1:-changed}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
O=gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests/test_gpu_native_sharded.py tests/test_c_caller.py tests/test_gpu_lde3.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_a.log 2>&1 || { echo "pytest a failed"; grep -E "FAIL|Error" $O/pytest_a.log | head; tail -30 $O/pytest_a.log; exit 1; }
tail -2 $O/pytest_a.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_full.log 2>&1 || { echo "pytest full failed"; grep -E "FAIL|Error" $O/pytest_full.log | head; tail -30 $O/pytest_full.log; exit 1; }
grep -E "PASS|passed|failed" $O/pytest_full.log | tail -12
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
python3 -c "
import json;l=[json.loads(x) for x in open('$O/bench.log') if x.startswith('{')][-1]
print({k:l.get(k) for k in ('ms_per_step','native_ms_per_step','verified','phase_ms','native_phase_ms')})"
