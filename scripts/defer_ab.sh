set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5ze && export TMPDIR=/tmp
for i in 1 2; do
  for d in 0 99; do
    BJ_EXPERIMENTS=1 BJ_LEAVES_DEFER=$d timeout -k 10 200 python3 -u tools/shard_compute_probe.py C3:2 C3:4 C3:8 > gpurun_out/r5ze/defer${d}_$i.log 2>&1 || { echo "probe d=$d rc=$?"; tail -5 gpurun_out/r5ze/defer${d}_$i.log; exit 1; }
    echo "d=$d run $i: $(python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1])['per_rank_compute'];print({k:(v['ms_per_rank'],v['phase_ms']) for k,v in d.items()})" gpurun_out/r5ze/defer${d}_$i.log)"
  done
done
