# Five default bench lines back to back on one box (box-to-box and run-to-run spread).
# usage: bash scripts/spread.sh TAG
set -u
TAG=${1:-spread}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
for i in 1 2 3 4 5; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/$TAG/c3_run$i.log 2>&1 || { echo "run $i failed"; tail -5 gpurun_out/$TAG/c3_run$i.log; exit 1; }
  python3 -c "import json,sys;l=[x for x in open(sys.argv[1]) if x.startswith('{')][-1];d=json.loads(l);print(sys.argv[2], round(d['ms_per_step'],2), round(d['native_ms_per_step'],2), {k:round(v,2) for k,v in d['phase_ms'].items()}, d['verified'])" gpurun_out/$TAG/c3_run$i.log $i
done
