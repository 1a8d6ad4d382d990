# Kernel trace of the per-rank compute of the G-way commit (exchange stubbed out,
# tools/shard_compute_probe.py): C3 at G = 1, 4, 8, one rocprofv3 --kernel-trace run each, so
# tools/shard_trace_summary.py can attribute what a rank pays above 1/G of the one-GPU commit.
# usage: bash scripts/shard_trace.sh TAG
set -u
TAG=${1:-shard_trace}
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
for G in 1 4 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/G$G -o run -- python3 tools/shard_compute_probe.py C3:$G > $OUT/probe_G$G.log 2>&1 || { echo "probe G=$G rc=$?"; tail -5 $OUT/probe_G$G.log; exit 1; }
  echo "G=$G $(grep -o '"ms_per_rank": [0-9.]*' $OUT/probe_G$G.log | head -1)"
done
