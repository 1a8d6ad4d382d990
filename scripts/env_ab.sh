# A/B of an environment knob on the stubbed per-rank probe (tools/shard_compute_probe.py),
# alternated three times on one box.  usage: bash scripts/env_ab.sh TAG VAR VALUE_A VALUE_B CFG...
# (an empty value leaves VAR unset)
set -u
TAG=$1; VAR=$2; A=$3; B=$4; shift 4
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
# the library reads its experiment knobs only under this gate (bj_internal.hpp, ABI 2.6)
export BJ_EXPERIMENTS=1
for i in 1 2 3; do
  for V in "$A" "$B"; do
    N=${V:-unset}
    if [ -n "$V" ]; then export $VAR=$V; else unset $VAR; fi
    timeout -k 10 200 python3 -u tools/shard_compute_probe.py "$@" > gpurun_out/$TAG/probe_${N}_$i.log 2>&1 || { echo "probe $N rc=$?"; tail -5 gpurun_out/$TAG/probe_${N}_$i.log; exit 1; }
    echo "$VAR=$N run $i: $(python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1])['per_rank_compute']
print({k:(v['ms_per_rank'],v['phase_ms']) for k,v in d.items()})" gpurun_out/$TAG/probe_${N}_$i.log)"
  done
done
unset $VAR
