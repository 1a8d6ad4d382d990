#!/bin/bash
# End-of-round GPU pass: every GPU test, the default bench line (with the CPU baseline), the
# N > 1 path launched both by torchrun and by bench.py itself (gloo rehearsal, ranks share the
# card), and a kernel trace of the default bench.  usage: bash scripts/final_check.sh TAG
set -u
TAG=${1:-final}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
O=gpurun_out/$TAG
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u bench.py > $O/bench_default.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-300
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --config C2 --steps 2 --warmup 1 > $O/torchrun2_C2.log 2>&1 || { echo "torchrun x2 failed"; tail -20 $O/torchrun2_C2.log; exit 1; }
grep '"metric"' $O/torchrun2_C2.log | cut -c1-200
timeout -k 10 300 python -u bench.py --gpus 4 --dist-backend gloo --config C2 --steps 2 --warmup 1 > $O/self4_C2.log 2>&1 || { echo "self-launch x4 failed"; tail -20 $O/self4_C2.log; exit 1; }
grep '"metric"' $O/self4_C2.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-native-base > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
echo done
