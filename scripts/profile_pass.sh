# Evidence pass for the C3 bench: a kernel-trace stats run, one PMC pass per counter group (HBM
# fetch, HBM write, SQ issue), the PMC summary restamped from those passes, and then the default
# bench line (with the CPU baseline), so that the line quotes the fresh traffic figures.
# The restamped profiles/pmc_summary.json is copied to gpurun_out/prof_TAG/ to be committed.
# usage: bash scripts/profile_pass.sh TAG
set -u
TAG=${1:-r4}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="python3 bench.py --config C3 --no-cpu-baseline --no-native-base"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B --steps 3 --warmup 1 > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $OUT/trace.log; exit 1; }
echo trace ok
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $B --steps 1 --warmup 0 > $OUT/fetch.log 2>&1 || { echo "fetch rc=$?"; tail -5 $OUT/fetch.log; exit 1; }
echo fetch ok
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $B --steps 1 --warmup 0 > $OUT/write.log 2>&1 || { echo "write rc=$?"; tail -5 $OUT/write.log; exit 1; }
echo write ok
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- $B --steps 1 --warmup 0 > $OUT/sq.log 2>&1 || { echo "sq rc=$?"; tail -5 $OUT/sq.log; exit 1; }
echo sq ok
python3 tools/pmc_summary.py $OUT --config C3 > $OUT/pmc_summary.log 2>&1 || { echo "pmc_summary rc=$?"; tail -5 $OUT/pmc_summary.log; exit 1; }
cp profiles/pmc_summary.json $OUT/pmc_summary.json
echo pmc summary restamped
timeout -k 10 500 python3 bench.py > $OUT/bench_default.log 2>&1 || { echo "bench rc=$?"; tail -5 $OUT/bench_default.log; exit 1; }
tail -1 $OUT/bench_default.log | cut -c1-300
