set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4l && export TMPDIR=/tmp
timeout -k 10 300 python -u tools/lde_overlap_ab.py C3 3 5 0 128 64 32 64h 32h > gpurun_out/r4l/overlap_ab.log 2>&1 || { echo "overlap failed"; tail -20 gpurun_out/r4l/overlap_ab.log; exit 1; }
grep '^{' gpurun_out/r4l/overlap_ab.log
