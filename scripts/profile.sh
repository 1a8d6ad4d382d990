#!/bin/bash
# rocprofv3 evidence for the C3 bench: the default bench line (with the CPU baseline), a
# kernel-trace stats run, one PMC pass per counter group, the FETCH_SIZE / WRITE_SIZE
# calibration on known byte counts (tools/fetch_calibration.hip), the per-rank compute probe,
# and (when built) the butterfly and power-of-two DFT microbenchmarks.
# usage: bash scripts/profile.sh TAG
set -u
TAG=${1:-r2}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 500 python3 bench.py > $OUT/bench_default.log 2>&1 || { echo "bench rc=$?"; tail -5 $OUT/bench_default.log; exit 1; }
tail -1 $OUT/bench_default.log
B="python3 bench.py --config C3 --no-cpu-baseline --no-native-base"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B --steps 3 --warmup 1 > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $OUT/trace.log; exit 1; }
echo trace ok
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $B --steps 1 --warmup 0 > $OUT/fetch.log 2>&1 || { echo "fetch rc=$?"; tail -5 $OUT/fetch.log; exit 1; }
echo fetch ok
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $B --steps 1 --warmup 0 > $OUT/write.log 2>&1 || { echo "write rc=$?"; tail -5 $OUT/write.log; exit 1; }
echo write ok
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- $B --steps 1 --warmup 0 > $OUT/sq.log 2>&1 || { echo "sq rc=$?"; tail -5 $OUT/sq.log; exit 1; }
echo sq ok
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/cal_fetch -o run -- ./tools/fetch_calibration > $OUT/cal_fetch.log 2>&1 || { echo "cal fetch rc=$?"; tail -5 $OUT/cal_fetch.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/cal_write -o run -- ./tools/fetch_calibration > $OUT/cal_write.log 2>&1 || { echo "cal write rc=$?"; tail -5 $OUT/cal_write.log; exit 1; }
echo calibration ok
PROBE_INTERFERE=1 timeout -k 10 400 python3 tools/shard_compute_probe.py > $OUT/shard_compute.log 2>&1 || { echo "probe rc=$?"; tail -5 $OUT/shard_compute.log; exit 1; }
tail -1 $OUT/shard_compute.log
if [ -x tools/pow2_bench ] && [ -x tools/bfly_bench ]; then
  timeout -k 10 120 ./tools/bfly_bench > $OUT/bfly_bench.log 2>&1 || { echo "bfly rc=$?"; exit 1; }
  timeout -k 10 120 ./tools/pow2_bench > $OUT/pow2_bench.log 2>&1 || { echo "pow2 rc=$?"; exit 1; }
  echo microbench ok
fi
echo done
