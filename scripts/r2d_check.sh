cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_native_sharded.py tests/test_gpu_rccl.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r2d.log 2>&1 && tail -2 gpurun_out/pytest_r2d.log && \
timeout -k 10 300 python -u bench.py --native --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_native_r2d.log 2>&1 && tail -1 gpurun_out/bench_native_r2d.log | cut -c1-900 && \
timeout -k 10 300 python -u bench.py --gpus 4 --dist-backend gloo --config C2 --steps 2 --warmup 1 > gpurun_out/bench_gloo4_r2d.log 2>&1 && tail -1 gpurun_out/bench_gloo4_r2d.log | cut -c1-1200
