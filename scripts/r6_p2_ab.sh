# Round 6: a Poseidon2 change (the half-reduced hand-off, r6a; the M4 blocks, r6d).  Parity first (permutation KATs, leaves, the
# proof.json paths, commits, the C3 golden cap), then the leaf kernel alone and the C3 commit,
# each alternated 3x against the previous library (era-boojum_amd/boojum_amd/libboojum_mi355x.so.old,
# tools/leaf_bench_prod_old).  usage: bash scripts/r6_p2_ab.sh TAG
set -u
TAG=${1:-r6a}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
O=gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "permutation or hash_into or proof_json or merkle or leaves or witness_commit or lde_commit_ex" > $O/pytest_parity.log 2>&1 \
  || { echo "pytest parity failed"; tail -30 $O/pytest_parity.log; exit 1; }
tail -1 $O/pytest_parity.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "fullsize_properties and C3" > $O/pytest_c3.log 2>&1 || { echo "pytest C3 failed"; tail -30 $O/pytest_c3.log; exit 1; }
tail -1 $O/pytest_c3.log
for V in old new old new old new; do
  B=tools/leaf_bench_prod; [ $V = old ] && B=tools/leaf_bench_prod_old
  timeout -k 10 120 $B 24 5 $V >> $O/leaf_bench.log 2>&1 || { echo "leaf bench $V failed"; tail -5 $O/leaf_bench.log; exit 1; }
done
cat $O/leaf_bench.log
bash scripts/ab_lib.sh $TAG C3
