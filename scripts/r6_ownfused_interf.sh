# Round 6: the own-column fusion beside the RCCL-shaped stand-in exchange (PROBE_INTERFERE=1:
# paced copies on the exchange stream), BJ_LDE_OWN_FUSED=0 against 1, alternated twice, C3 at
# G = 2 and 4 (the all-gather cases).  usage: bash scripts/r6_ownfused_interf.sh TAG
set -u
TAG=${1:-r6g}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp BJ_EXPERIMENTS=1 PROBE_INTERFERE=1
for i in 1 2; do
  for V in 0 1; do
    BJ_LDE_OWN_FUSED=$V timeout -k 10 500 python3 -u tools/shard_compute_probe.py C3:2 C3:4 > gpurun_out/$TAG/interf_${V}_$i.log 2>&1 || { echo "probe $V rc=$?"; tail -5 gpurun_out/$TAG/interf_${V}_$i.log; exit 1; }
    python3 -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
d=d.get('per_rank_compute',d)
print(sys.argv[2], {c:{k:(v['ms'] if isinstance(v,dict) and 'ms' in v else None) for k,v in d[c]['interference'].items() if k!='phase_events_in_timed_calls'} for c in d})" gpurun_out/$TAG/interf_${V}_$i.log "own_fused=$V run $i"
  done
done
