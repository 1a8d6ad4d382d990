# Full GPU pass: smoke(), every GPU test, the bench at C1 / C2 / C5 / C4, and the N > 1
# launch paths (torchrun x2 and self-launched x4 over the gloo rehearsal transport, C2).
# usage: bash scripts/full_pass.sh TAG
set -u
TAG=${1:-r4full}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
O=gpurun_out/$TAG
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for C in C1 C2 C5 C4; do
  S=5; [ $C = C4 ] && S=3
  timeout -k 10 400 python -u bench.py --config $C --steps $S --warmup 1 --no-cpu-baseline --no-native-base > $O/bench_$C.log 2>&1 || { echo "bench $C failed"; tail -5 $O/bench_$C.log; exit 1; }
  python3 -c "import json,sys;l=[x for x in open(sys.argv[1]) if x.startswith('{')][-1];d=json.loads(l);print(sys.argv[2], round(d['ms_per_step'],2), '%.3e' % d['value'], {k:round(v,2) for k,v in d['phase_ms'].items()}, d['verified'])" $O/bench_$C.log $C
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --config C2 --steps 2 --warmup 1 > $O/torchrun2_C2.log 2>&1 || { echo "torchrun x2 failed"; tail -20 $O/torchrun2_C2.log; exit 1; }
grep '"metric"' $O/torchrun2_C2.log | cut -c1-160
timeout -k 10 300 python -u bench.py --gpus 4 --dist-backend gloo --config C2 --steps 2 --warmup 1 > $O/self4_C2.log 2>&1 || { echo "self-launch x4 failed"; tail -20 $O/self4_C2.log; exit 1; }
grep '"metric"' $O/self4_C2.log | cut -c1-160
grep -o '"verified": [a-z]*' $O/self4_C2.log $O/torchrun2_C2.log
echo done
