"""bench.py --gpus N without an external launcher starts N rank processes itself (the parent
never touches a GPU) and returns the first failing rank's exit code after stopping the others.
On a machine without a GPU every rank fails at its device selection, which exercises exactly
that failure path: the parent must return non-zero promptly, not hang."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_self_launch_reports_a_failing_rank():
    import torch
    if torch.cuda.is_available():
        import pytest
        pytest.skip("needs a machine without a GPU (every rank must fail)")
    t0 = time.time()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "C1", "--steps",
                        "1", "--warmup", "0", "--no-cpu-baseline"], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode != 0
    assert "No HIP GPUs" in r.stderr or "CUDA" in r.stderr or "HIP" in r.stderr
    assert time.time() - t0 < 240


def test_rank_count_must_match_world_size():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--config", "C1"], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode != 0 and "WORLD_SIZE=2" in (r.stderr + r.stdout)
