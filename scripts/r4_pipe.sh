set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4f && export TMPDIR=/tmp
O=gpurun_out/r4f
timeout -k 10 300 python -u tools/pipe_ab.py C3 3 6 serial pipe pipe+s2hi pipe+s2lo pipe+w4 > $O/pipe_ab.log 2>&1 || { echo "pipe_ab failed"; tail -20 $O/pipe_ab.log; exit 1; }
grep '^{' $O/pipe_ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/pipe_ab.py C3 1 2 pipe > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
echo trace ok
