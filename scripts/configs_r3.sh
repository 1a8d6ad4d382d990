#!/bin/bash
# The bench at every BASELINE config on one GPU (C1, C2, C4, C5) and the N > 1 launch paths
# (torchrun x2 and self-launched x4 over the gloo rehearsal transport, ranks sharing the card).
# usage: bash scripts/configs_r3.sh TAG
set -u
TAG=${1:-cfg}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
O=gpurun_out/$TAG
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
