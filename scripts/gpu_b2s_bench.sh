#!/bin/bash
# Blake2s256-tree commits: C3 and C5 benches, kernel trace of C3, PMC traffic of the leaf kernel.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/b2s
mkdir -p $OUT
timeout -k 10 300 python3 bench.py --config C3 --hasher blake2s --steps 5 --warmup 2 --cpu-sample-log-n 20 > $OUT/bench_c3.log 2>&1 || { echo "c3 rc=$?"; tail -5 $OUT/bench_c3.log; exit 1; }
tail -1 $OUT/bench_c3.log
timeout -k 10 300 python3 bench.py --config C5 --hasher blake2s --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_c5.log 2>&1 || { echo "c5 rc=$?"; tail -5 $OUT/bench_c5.log; exit 1; }
tail -1 $OUT/bench_c5.log
timeout -k 10 300 python3 bench.py --config C5 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_c5_p2.log 2>&1 || { echo "c5p2 rc=$?"; tail -5 $OUT/bench_c5_p2.log; exit 1; }
tail -1 $OUT/bench_c5_p2.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --config C3 --hasher blake2s --steps 3 --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $OUT/trace.log; exit 1; }
echo trace ok
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py --config C3 --hasher blake2s --steps 1 --warmup 0 --no-cpu-baseline > $OUT/fetch.log 2>&1 || { echo "fetch rc=$?"; tail -5 $OUT/fetch.log; exit 1; }
echo fetch ok
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/write -o run -- python3 bench.py --config C3 --hasher blake2s --steps 1 --warmup 0 --no-cpu-baseline > $OUT/write.log 2>&1 || { echo "write rc=$?"; tail -5 $OUT/write.log; exit 1; }
echo write ok
