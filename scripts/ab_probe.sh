# A/B of two builds of the library on one box through the per-rank compute probe
# (tools/shard_compute_probe.py), alternated; the previous build at
# era-boojum_amd/boojum_amd/libboojum_mi355x.so.old (swapped in and out, as scripts/ab_lib.sh).
# usage: bash scripts/ab_probe.sh TAG [config[:G] ...]
set -u
TAG=${1:-abp}
shift
CFGS=${*:-C3:8}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
O=gpurun_out/$TAG
L=era-boojum_amd/boojum_amd/libboojum_mi355x.so
cp $L $L.new
for V in old new old new; do
  cp $L.$V $L
  timeout -k 10 200 python3 -u tools/shard_compute_probe.py $CFGS > $O/probe_$V.log 2>&1 || { echo "probe $V failed"; tail -5 $O/probe_$V.log; cp $L.new $L; exit 1; }
  grep '^{"C' $O/probe_$V.log | sed "s/^/$V /" | tee -a $O/probe_ab.log
done
cp $L.new $L
