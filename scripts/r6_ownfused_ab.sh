# Round 6: G <= D ranks fuse their own columns' inverse tail into their cosets' forward pass
# (bj::lde_own_shard).  Parity (the collective at G = 1..8 incl. the new cases, the knob test, the
# C3 collective golden caps, the C4 one-coset-per-rank split), then the stubbed per-rank call at
# C3 G = 2 / 4 and C4 G = 8 with BJ_LDE_OWN_FUSED=0 against 1, alternated 3x.
# usage: bash scripts/r6_ownfused_ab.sh TAG
set -u
TAG=${1:-r6f}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
O=gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests/test_gpu_native_sharded.py tests/test_gpu_fullsize.py -m gpu -x -q \
  --timeout 400 --timeout-method thread -k "local_ranks or env_knobs or c3_collective or c4_one_coset or c3_full_size" \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash scripts/env_ab.sh ${TAG}_ab BJ_LDE_OWN_FUSED 0 1 C3:2 C3:4 C4:8
