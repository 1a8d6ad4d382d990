"""bench.py --gpus N without an external launcher starts N rank processes itself (the parent
never touches a GPU) and returns the first failing rank's exit code after stopping the others.
On a machine without a GPU every rank fails at its device selection, which exercises exactly
that failure path: the parent must return non-zero promptly, not hang."""
import json
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


def _bench(args, **env_extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra)
    return subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, stdout=subprocess.PIPE,
                            stderr=subprocess.PIPE, text=True)


def test_hung_rank_ends_the_job_inside_the_deadline():
    """A rank that never reaches its rendezvous: the parent's deadline stops every rank (SIGTERM,
    then SIGKILL) and prints one JSON error line naming the ranks alive and their last phases."""
    t0 = time.time()
    p = _bench(["--gpus", "2", "--launch-check", "--timeout", "15"], BJ_BENCH_TEST_HANG_RANK="1")
    out, err = p.communicate(timeout=120)
    elapsed = time.time() - t0
    assert p.returncode == 124, (out, err)
    line = json.loads(out.strip().splitlines()[-1])
    assert "deadline" in line["error"]
    assert line["ranks_alive"] == [0, 1]
    assert line["last_phase"]["1"] == "test-hang"
    assert line["last_phase"]["0"] == "init"
    assert 15 <= elapsed < 60


def test_two_self_launched_jobs_do_not_collide():
    """Two 4-rank jobs started together on one host rendezvous through their own file stores."""
    jobs = [_bench(["--gpus", "4", "--launch-check", "--timeout", "120"]) for _ in range(2)]
    for p in jobs:
        out, err = p.communicate(timeout=180)
        assert p.returncode == 0, err
        line = json.loads(out.strip().splitlines()[-1])
        assert line == {"launch_check": "ok", "n_gpus": 4, "rank_sum": 10, "rendezvous": "file"}


def test_rank_watchdog_under_an_external_launcher():
    """Under torchrun-style env (no parent deadline) a hung rank still ends itself (exit 124)."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", BJ_BENCH_TEST_HANG_RANK="0")
    env.pop("BJ_BENCH_INIT", None)
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--launch-check", "--timeout", "5"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 124 and "deadline passed in phase 'test-hang'" in r.stderr
    assert time.time() - t0 < 60


def test_world_record_from_gathered_infos():
    """The N > 1 line's transport record (bench.world_record) from bj_comm_check_world's gathered
    bj_comm_info_t records: RCCL's own count and ranks, devices, bus ids, hosts."""
    import bench
    infos = [{"kind": "rccl", "world": 4, "rank": r, "transport_count": 4, "transport_rank": r, "device": r,
              "pci_bus_id": "0000:%02x:00.0" % (0x10 * (r + 1)), "host": "node0"} for r in range(4)]
    rec = bench.world_record(infos, "nccl", "")
    assert rec["backend"] == "rccl" and rec["count"] == 4 and rec["ranks"] == [0, 1, 2, 3]
    assert rec["devices"] == [0, 1, 2, 3] and rec["distinct_devices"] == 4 and rec["check"] == "ok"
    assert rec["hosts"] == ["node0"]
    # ranks that share a device (as the gloo rehearsal's do) count once; a failed check keeps its message
    shared = [dict(i, device=0, pci_bus_id="0000:10:00.0") for i in infos]
    rec = bench.world_record(shared, "gloo", "ranks 0 and 1 share device 0")
    assert rec["backend"] == "gloo (callback transport)" and rec["distinct_devices"] == 1
    assert rec["check"] == "ranks 0 and 1 share device 0"


def test_link_record_schema():
    """The N > 1 line's "link" object (bench.link_record): one exchange of the run's own kind and
    size, timed on every rank before the timed region; min / max over ranks.  The exchange shapes
    are bj_sharded_commit_d's: C3 at G = 4 all-gathers 2 GiB per rank block (6 GiB
    from peers), at G = 8 > D one all-to-all of 512 MiB per destination (3.5 GiB from peers)."""
    import bench
    assert bench.exchange_shape(256, 22, 2, 4) == ("all_gather", 2 << 30)
    assert bench.exchange_shape(256, 22, 2, 8) == ("all_to_all", 512 << 20)
    assert bench.exchange_shape(256, 23, 3, 8) == ("all_gather", 2 << 30)           # C4: G = D
    assert bench.exchange_shape(128, 20, 1, 8) == ("all_to_all", 32 << 20)          # C2 at G = 8
    assert bench.exchange_shape(16, 18, 3, 8, log_commit_cosets=1) == ("all_gather", 4 << 20)
    assert bench.exchange_shape(16, 18, 2, 8, log_commit_cosets=1) == ("all_to_all", 8 * (1 << 16) * 2 * 2)
    rec = bench.link_record("all_to_all", 512 << 20, 8, [30.0, 28.0, 35.0, 29.0, 28.5, 31.0, 30.5, 29.5], "nccl")
    assert set(rec) >= {"kind", "bytes_per_rank", "ms", "gbs_per_rank"}
    assert rec["kind"] == "all_to_all" and rec["bytes_per_rank"] == 7 * (512 << 20)
    assert rec["ms"] == [28.0, 35.0]
    lo, hi = rec["gbs_per_rank"]
    assert abs(hi - 7 * (512 << 20) / 28.0 / 1e6) < 1e-9 and lo < hi
    assert rec["transport"] == "rccl" and "note" not in rec
    json.dumps(rec)
    rec = bench.link_record("all_gather", 1 << 20, 2, [5.0, 6.0], "gloo")
    assert rec["bytes_per_rank"] == 1 << 20 and "not a link rate" in rec["note"]
