# Run-to-run spread of the default C3 line on one box (five runs, CPU baseline off), and the
# other configs' verified lines.  usage: bash scripts/spread.sh TAG
set -u
TAG=${1:-spread}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
for i in 1 2 3 4 5; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/$TAG/c3_$i.log 2>&1 || { echo "run $i failed"; tail -3 gpurun_out/$TAG/c3_$i.log; exit 1; }
  echo "C3 run $i $(python3 -c "import json;l=[x for x in open('gpurun_out/$TAG/c3_$i.log') if x.startswith('{')][-1];d=json.loads(l);print(round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['phase_ms'].items()},d['verified'])")"
done
for C in C2 C5; do
  timeout -k 10 200 python -u bench.py --config $C --no-cpu-baseline > gpurun_out/$TAG/$C.log 2>&1 || { echo "$C failed"; exit 1; }
  echo "$C $(python3 -c "import json;l=[x for x in open('gpurun_out/$TAG/$C.log') if x.startswith('{')][-1];d=json.loads(l);print(round(d['ms_per_step'],3),d['verified'])")"
done
