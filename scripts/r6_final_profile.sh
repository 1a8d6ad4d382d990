# Round 6's profile pass on the final library: the C3 kernel-trace stats, the PMC passes (HBM
# fetch / write, SQ issue) restamping profiles/pmc_summary.json, the default bench line with the
# CPU baseline (scripts/profile_pass.sh), then the kernel traces of the stubbed per-rank call at
# G = 1 / 4 / 8 (scripts/shard_trace.sh).  usage: bash scripts/r6_final_profile.sh TAG
set -u
TAG=${1:-r6prof}
bash scripts/profile_pass.sh $TAG || exit 1
bash scripts/shard_trace.sh ${TAG}_shard_trace || exit 1
cd "$GRAFT_REPO_ROOT"
python3 tools/shard_trace_summary.py gpurun_out/${TAG}_shard_trace --json gpurun_out/${TAG}_shard_trace/summary.json \
  > gpurun_out/${TAG}_shard_trace/summary.txt 2>&1 || { echo "summary failed"; tail -5 gpurun_out/${TAG}_shard_trace/summary.txt; exit 1; }
grep "span" gpurun_out/${TAG}_shard_trace/summary.txt
