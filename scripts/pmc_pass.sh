#!/bin/bash
# PMC refresh for the C3 bench on the current library: a kernel-trace stats run and one PMC pass
# per counter group (FETCH_SIZE, WRITE_SIZE, SQ), each under its own time limit; then
# tools/pmc_summary.py gpurun_out/prof_TAG turns them into profiles/pmc_summary.json (on the CPU).
# usage: bash scripts/pmc_pass.sh TAG
set -u
TAG=${1:-r3}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="python3 bench.py --config C3 --no-cpu-baseline --no-native-base"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B --steps 3 --warmup 1 > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $OUT/trace.log; exit 1; }
tail -1 $OUT/trace.log | cut -c1-300
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $B --steps 1 --warmup 0 > $OUT/fetch.log 2>&1 || { echo "fetch rc=$?"; tail -5 $OUT/fetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $B --steps 1 --warmup 0 > $OUT/write.log 2>&1 || { echo "write rc=$?"; tail -5 $OUT/write.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- $B --steps 1 --warmup 0 > $OUT/sq.log 2>&1 || { echo "sq rc=$?"; tail -5 $OUT/sq.log; exit 1; }
echo pmc ok
