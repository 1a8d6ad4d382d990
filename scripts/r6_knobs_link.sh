# Round 6: the experiment-knob gate, the world check's invalid-record path and the N > 1 line's
# link probe, on one card.  usage: bash scripts/r6_knobs_link.sh TAG
set -u
TAG=${1:-r6b}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
O=gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_native_sharded.py tests/test_gpu_lde3.py tests/test_gpu_parity.py \
  tests/test_c_caller.py tests/test_gpu_rccl.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "env_knobs or two_pass or one_per_lane or errors_are_loud or c_caller or rccl or comm_info" > $O/pytest.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for CFG in C2 C3; do
  timeout -k 10 500 python -u bench.py --gpus 8 --dist-backend gloo --config $CFG --steps 2 --warmup 1 \
    --no-cpu-baseline --timeout 420 > $O/self8_$CFG.log 2>&1 || { echo "self8 $CFG failed"; tail -5 $O/self8_$CFG.log; exit 1; }
  python3 -c "
import json;l=[json.loads(x) for x in open('$O/self8_$CFG.log') if x.startswith('{')][-1]
print('$CFG', l.get('verified'), json.dumps(l.get('link')))"
done
timeout -k 10 300 python -u bench.py --gpus 4 --dist-backend gloo --config C2 --steps 2 --warmup 1 \
  --no-cpu-baseline --timeout 240 > $O/self4_C2.log 2>&1 || { echo "self4 failed"; tail -5 $O/self4_C2.log; exit 1; }
python3 -c "
import json;l=[json.loads(x) for x in open('$O/self4_C2.log') if x.startswith('{')][-1]
print('C2 x4', l.get('verified'), json.dumps(l.get('link')))"
