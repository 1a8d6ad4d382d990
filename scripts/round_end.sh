# Round-end pass: smoke(), the N = 1 native-collective bench, then scripts/final_check.sh
# (every GPU test, the default bench, torchrun and self-launched N > 1 rehearsals, kernel trace).
# usage: bash scripts/round_end.sh TAG
set -u
TAG=${1:-end}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
timeout -k 10 300 python3 -u bench.py --native --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/bench_native.log 2>&1 || { echo "native bench failed"; tail -20 gpurun_out/$TAG/bench_native.log; exit 1; }
grep '"metric"' gpurun_out/$TAG/bench_native.log | cut -c1-220
bash scripts/final_check.sh $TAG
