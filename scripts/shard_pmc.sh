# HBM traffic of the per-rank kernels of the stubbed G-way call (tools/shard_compute_probe.py
# C3:8 by default): a kernel trace, then FETCH_SIZE and WRITE_SIZE in passes of their own.
# usage: bash scripts/shard_pmc.sh TAG [probe args]
set -u
TAG=${1:-shard_pmc}
shift || true
ARGS=${*:-C3:8}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
O=gpurun_out/$TAG
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/shard_compute_probe.py $ARGS > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
echo trace ok
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 tools/shard_compute_probe.py $ARGS > $O/fetch.log 2>&1 || { echo "fetch rc=$?"; tail -5 $O/fetch.log; exit 1; }
echo fetch ok
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 tools/shard_compute_probe.py $ARGS > $O/write.log 2>&1 || { echo "write rc=$?"; tail -5 $O/write.log; exit 1; }
echo write ok
