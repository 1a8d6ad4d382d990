#!/bin/bash
# Node-level A/B: one node per quad of lanes for the small levels (default) against one node per
# lane with the one-workgroup tail (BJ_NODE_Q4_MAX=0), alternated, C1 / C5 / C2 / C3; first the
# Merkle, commit and sharded GPU tests.  usage: bash scripts/ab_nodes.sh TAG
set -u
TAG=${1:-nodes}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
O=gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest.log | head; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
summ() { python3 -c "import json,sys;l=[x for x in open(sys.argv[1]) if x.startswith('{')][-1];d=json.loads(l);print(round(d['ms_per_step'],3),{k:round(v,3) for k,v in d['phase_ms'].items()},d['verified'])" $1; }
for C in C1 C5 C2 C3; do
  S=20; [ $C = C3 ] && S=6
  for i in 1 2; do
    for V in q4 lane; do
      if [ $V = lane ]; then E="BJ_NODE_Q4_MAX=0"; else E="BJ_NODE_Q4_MAX=32768"; fi
      env $E timeout -k 10 300 python3 -u bench.py --config $C --steps $S --warmup 2 --no-cpu-baseline --no-native-base > $O/${C}_${V}_$i.log 2>&1 || { echo "bench $C $V failed"; tail -5 $O/${C}_${V}_$i.log; exit 1; }
      echo "$C $V: $(summ $O/${C}_${V}_$i.log)"
    done
  done
done
echo done
