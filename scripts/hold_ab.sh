# Exchange hold (BJ_XCHG_HOLD, collective.hip) under the RCCL-shaped stand-in
# (tools/shard_compute_probe.py PROBE_INTERFERE=1), alternated; then the sharded GPU tests under
# each hold.  usage: bash scripts/hold_ab.sh TAG
set -u
TAG=${1:-hold}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
for i in 1 2; do
  for h in 0 1 2; do
    BJ_XCHG_HOLD=$h PROBE_INTERFERE=1 timeout -k 10 200 python3 -u tools/shard_compute_probe.py C3:4 C3:8 > gpurun_out/$TAG/hold${h}_$i.log 2>&1 || { echo "probe h=$h rc=$?"; tail -5 gpurun_out/$TAG/hold${h}_$i.log; exit 1; }
    python3 - gpurun_out/$TAG/hold${h}_$i.log $h $i <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])["per_rank_compute"]
out = []
for k, v in d.items():
    it = v["interference"]
    out.append("%s stub %.2f 16ch64 %s 32ch64 %s burst %s" % (k, it["stubbed"]["ms"], it[[n for n in it if n.startswith("paced_16ch") ][0]]["ms"],
                                                           it[[n for n in it if n.startswith("paced_32ch")][0]]["ms"], it["burst_32ch"]["ms"]))
print("h=%s run %s: %s" % (sys.argv[2], sys.argv[3], " | ".join(out)))
PY
  done
done
for h in 1 2; do
  BJ_XCHG_HOLD=$h timeout -k 10 400 python -u -m pytest tests/test_gpu_native_sharded.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/tests_hold$h.log 2>&1 || { echo "tests h=$h failed"; tail -20 gpurun_out/$TAG/tests_hold$h.log; exit 1; }
  echo "tests h=$h: $(tail -n 1 gpurun_out/$TAG/tests_hold$h.log)"
done
