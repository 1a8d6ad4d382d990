# Round 6 per-rank evidence on the current library: the kernel traces of the stubbed call at
# G = 1 / 4 / 8 (scripts/shard_trace.sh), then C3 at G = 8 beside the RCCL-shaped stand-in
# exchange (PROBE_INTERFERE=1), twice.  usage: bash scripts/r6_shard_evidence.sh TAG
set -u
TAG=${1:-r6e}
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/$TAG
bash scripts/shard_trace.sh ${TAG}_shard_trace || exit 1
python3 tools/shard_trace_summary.py gpurun_out/${TAG}_shard_trace --json gpurun_out/${TAG}_shard_trace/summary.json > gpurun_out/${TAG}_shard_trace/summary.txt 2>&1 || { echo "summary failed"; tail -5 gpurun_out/${TAG}_shard_trace/summary.txt; exit 1; }
tail -12 gpurun_out/${TAG}_shard_trace/summary.txt
for i in 1 2; do
  PROBE_INTERFERE=1 timeout -k 10 500 python3 -u tools/shard_compute_probe.py C3:8 > gpurun_out/$TAG/interference_G8_$i.log 2>&1 || { echo "interference $i rc=$?"; tail -5 gpurun_out/$TAG/interference_G8_$i.log; exit 1; }
  python3 -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
d=d.get('per_rank_compute',d)['C3_G8']['interference']
print({k:(v['ms'] if isinstance(v,dict) and 'ms' in v else None) for k,v in d.items()})" gpurun_out/$TAG/interference_G8_$i.log
done
