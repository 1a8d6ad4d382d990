# Every bench config's line against its golden cap, the C3 Blake2s tree, and the power-of-two DFT check
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/cfg && export TMPDIR=/tmp
for C in C1 C2 C4 C5; do
  timeout -k 10 300 python -u bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/cfg/bench_$C.log 2>&1 || { echo "bench $C failed"; tail -5 gpurun_out/cfg/bench_$C.log; exit 1; }
  echo "$C $(python3 -c "import json;l=[x for x in open('gpurun_out/cfg/bench_$C.log') if x.startswith('{')][-1];d=json.loads(l);print(round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['phase_ms'].items()},d['verified'])")"
done
timeout -k 10 300 python -u bench.py --config C5 --hasher blake2s --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/cfg/bench_C5_b2s.log 2>&1 || { echo "bench C5 blake2s failed"; exit 1; }
grep -o '"verified": [a-z]*' gpurun_out/cfg/bench_C5_b2s.log
timeout -k 10 120 ./tools/pow2_bench > gpurun_out/cfg/pow2_bench.log 2>&1 || { echo "pow2 failed"; exit 1; }
tail -4 gpurun_out/cfg/pow2_bench.log
