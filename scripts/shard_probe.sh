# Per-rank compute of the G-way commit with the exchange stubbed out (tools/shard_compute_probe.py):
# C3 at G = 1, 2, 4, 8 and C4 at G = 8, phases inside the call.  usage: bash scripts/shard_probe.sh TAG
set -u
TAG=${1:-probe}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
timeout -k 10 500 python3 -u tools/shard_compute_probe.py > gpurun_out/$TAG/shard_compute.log 2>&1 || { echo "probe rc=$?"; tail -20 gpurun_out/$TAG/shard_compute.log; exit 1; }
tail -12 gpurun_out/$TAG/shard_compute.log
