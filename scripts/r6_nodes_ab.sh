# Round 6: the small subtree levels up to 8 per launch (node_levels_q4_kernel) and two chunks per
# leaf grid in the collective.  Parity (trees of 2 .. 2^18 leaves, every node form, the
# collective's subtrees at G = 1..8 and its knobs, the C3 cap), the C3 commit alternated against
# the previous library (libboojum_mi355x.so.old), then same-binary knob A/Bs of the stubbed
# per-rank call at G = 1 / 4 / 8 (BJ_NODE_FUSED=0, BJ_LEAVES_GROUP=1 restore the previous
# schedule).  usage: bash scripts/r6_nodes_ab.sh TAG
set -u
TAG=${1:-r6c}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
O=gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_native_sharded.py tests/test_gpu_fullsize.py \
  -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "merkle_tree or one_per_lane or native_sharded_commit or (fullsize_properties and C3) or c3_collective" \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash scripts/ab_lib.sh $TAG C3 || exit 1
bash scripts/env_ab.sh ${TAG}_fused BJ_NODE_FUSED 0 1 C3:1 C3:4 C3:8 || exit 1
bash scripts/env_ab.sh ${TAG}_group BJ_LEAVES_GROUP 1 2 C3:4 C3:8
