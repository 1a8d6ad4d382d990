#!/bin/bash
# N>1 bench path rehearsal on one GPU (gloo staging, ranks share the card): not a benchmark.
# Runs the driver's launch line shape at N = 2 and 4 (C2 and C3 geometry).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for spec in "2 C2" "4 C2" "4 C3"; do
    set -- $spec
    timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $1 --steps 2 --warmup 1 --config $2 --dist-backend gloo > gpurun_out/rehearse_$1_$2.log 2>&1 || { echo "rehearse N=$1 $2 rc=$?"; tail -30 gpurun_out/rehearse_$1_$2.log; exit 1; }
    echo "N=$1 $2: $(tail -1 gpurun_out/rehearse_$1_$2.log | cut -c1-300)"
done
