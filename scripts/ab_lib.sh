# A/B of two builds of the library on one box: copy the previous build to
# era-boojum_amd/boojum_amd/libboojum_mi355x.so.old first (it is swapped in and out).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab && export TMPDIR=/tmp
L=era-boojum_amd/boojum_amd/libboojum_mi355x.so
cp $L $L.new
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "lde or fft or transforms or fullsize or c2" > gpurun_out/ab/pytest.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/ab/pytest.log; exit 1; }
tail -1 gpurun_out/ab/pytest.log
for V in old new old new old new; do
  cp $L.$V $L
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab/bench_$V.log 2>&1 || { echo "bench $V failed"; tail -5 gpurun_out/ab/bench_$V.log; exit 1; }
  echo "$V $(python3 -c "import json;l=[x for x in open('gpurun_out/ab/bench_$V.log') if x.startswith('{')][-1];d=json.loads(l);print(round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['phase_ms'].items()},d['verified'])")"
done
cp $L.new $L
