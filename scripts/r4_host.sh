set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4g && export TMPDIR=/tmp
O=gpurun_out/r4g/host_resident.log
: > $O
for cfg in "20 128 1" "22 256 2"; do
  for mode in pageable pinned; do
    echo "== $cfg $mode" >> $O
    timeout -k 10 240 python3 -u tools/host_resident.py $cfg $mode >> $O 2>&1 || { echo "host_resident $cfg $mode rc=$?"; tail -5 $O; exit 1; }
  done
done
cat $O
