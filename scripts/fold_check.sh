set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4q && export TMPDIR=/tmp
O=gpurun_out/r4q
timeout -k 10 500 python -u -m pytest tests/test_gpu_native_sharded.py tests/test_c_caller.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python3 -u tools/shard_compute_probe.py C3 > $O/shard_compute.log 2>&1 || { echo "probe rc=$?"; tail -20 $O/shard_compute.log; exit 1; }
grep '"C3_G' $O/shard_compute.log | cut -c1-260
BJ_FUSED_FOLD=0 timeout -k 10 200 python3 -u tools/shard_compute_probe.py C3 > $O/shard_compute_nofuse.log 2>&1 || { echo "probe2 rc=$?"; exit 1; }
grep '"C3_G8' $O/shard_compute_nofuse.log | cut -c1-260
