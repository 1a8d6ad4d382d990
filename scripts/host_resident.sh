# The host-buffer boundary (bj_lde_commit_h, PCIe-inclusive) at C2 and C3, pageable and
# page-locked caller buffers.  usage: bash scripts/host_resident.sh TAG
set -u
TAG=${1:-host}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
O=gpurun_out/$TAG/host_resident.log
: > $O
for cfg in "20 128 1" "22 256 2"; do
  for mode in pageable pinned; do
    echo "== $cfg $mode" >> $O
    timeout -k 10 240 python3 -u tools/host_resident.py $cfg $mode >> $O 2>&1 || { echo "host_resident $cfg $mode rc=$?"; tail -5 $O; exit 1; }
  done
done
cat $O
