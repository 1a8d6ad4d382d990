# A/B of two library builds (.so.old vs .so.new, alternated twice) on the stubbed per-rank probe
# (tools/shard_compute_probe.py) for the configs given.  usage: bash scripts/ab_probe_libs.sh TAG CFG...
set -u
TAG=$1; shift
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
L=era-boojum_amd/boojum_amd/libboojum_mi355x.so
cp $L $L.new
for i in 1 2; do
  for V in old new; do
    cp $L.$V $L
    timeout -k 10 300 python3 -u tools/shard_compute_probe.py "$@" > gpurun_out/$TAG/probe_${V}_$i.log 2>&1 || { echo "probe $V failed"; tail -5 gpurun_out/$TAG/probe_${V}_$i.log; cp $L.new $L; exit 1; }
    echo "$V $(python3 -c "
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{') and 'per_rank_compute' not in l:
        d=json.loads(l); k=list(d)[0]; print(k, d[k]['ms_per_rank'], end='  ')
" gpurun_out/$TAG/probe_${V}_$i.log)"
  done
done
cp $L.new $L
