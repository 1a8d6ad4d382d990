# A/B of two builds of the library on one box, alternated: the previous build is expected at
# era-boojum_amd/boojum_amd/libboojum_mi355x.so.old (it is swapped in and out).
# usage: bash scripts/ab_lib.sh TAG [config]
set -u
TAG=${1:-ab}
CFG=${2:-C3}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
O=gpurun_out/$TAG
L=era-boojum_amd/boojum_amd/libboojum_mi355x.so
cp $L $L.new
for V in old new old new old new; do
  cp $L.$V $L
  timeout -k 10 200 python -u bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-native-base > $O/bench_$V.log 2>&1 || { echo "bench $V failed"; tail -5 $O/bench_$V.log; cp $L.new $L; exit 1; }
  cat $O/bench_$V.log >> $O/bench_all_$V.log
  echo "$V $(python3 -c "import json;l=[x for x in open('$O/bench_$V.log') if x.startswith('{')][-1];d=json.loads(l);print(round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['phase_ms'].items()},d['verified'])")"
done
cp $L.new $L
