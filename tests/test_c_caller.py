"""The C ABI driven from plain C (tests/c/c_caller.c), the way a Rust prover's FFI binds it:
host buffers, per-column FFT seam called concurrently from threads, TreeHasher, the
host-buffer witness commit and the error contract, each checked against the CPU oracle.

The non-GPU test only checks that the caller links against the product library; the GPU
tests run it (C1's geometry at two thread counts, a ragged column count, LDE x8)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "c", "c_caller")


def _need_bin():
    if not os.path.exists(BIN):
        pytest.fail("tests/c/c_caller is not built (run __graft_entry__.build())")


def test_c_caller_links_the_product_library():
    _need_bin()
    out = subprocess.run(["ldd", BIN], check=True, capture_output=True, text=True).stdout
    lines = {ln.split()[0]: ln for ln in out.splitlines() if "=>" in ln}
    assert "libboojum_mi355x.so" in lines and "not found" not in lines["libboojum_mi355x.so"], out
    assert "liboracle.so" in lines and "not found" not in lines["liboracle.so"], out


@pytest.mark.gpu
@pytest.mark.parametrize("log_n,cols,log_lde,cap,threads,log_k", [
    (16, 32, 1, 16, 8, 1),    # C1, seam called from 8 threads
    (12, 19, 2, 8, 3, 2),     # ragged leaf length (19 = 2 sponge blocks + 3)
    (10, 8, 3, 32, 1, 3),     # LDE x8, cap 32
    (14, 16, 3, 32, 4, 1),    # proof.json's shape ratio: LDE x8 (quotient degree), 2 cosets committed, cap 32
    (13, 16, 2, 16, 2, 0),    # LDE x4, one coset committed (G = 8 > D: the sender-side fold)
])
def test_c_caller(log_n, cols, log_lde, cap, threads, log_k):
    _need_bin()
    r = subprocess.run([BIN, str(log_n), str(cols), str(log_lde), str(cap), str(threads), str(log_k)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "c_caller ok" in r.stdout, r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("log_n,cols,log_lde,cap,threads,log_k", [
    (12, 16, 2, 16, 2, 2),    # D = 4: G = 2 all-gather (G < D), 4 (G = D), 8 all-to-all of sender folds (G > D)
    (13, 16, 3, 32, 2, 1),    # D = 8, k = 2 committed (proof.json's ratio): every block of k cosets
])
def test_c_caller_collective_over_rccl_api(log_n, cols, log_lde, cap, threads, log_k):
    """The collective commit through the library's RCCL code path at G = 2, 4, 8 ranks on one GPU
    (and the world check each N > 1 bench line carries: counts, ranks, duplicated device):
    the mock librccl.so.1 (tests/c/mock_rccl.cpp) gives RCCL's semantics for in-process ranks, so
    the in-place ncclAllGather offsets, the grouped ncclSend / ncclRecv pairing and their stream
    ordering are exercised as a multi-GPU run issues them; results checked against the oracle."""
    _need_bin()
    mock = os.path.join(ROOT, "tests", "c", "libmock_rccl.so")
    if not os.path.exists(mock):
        pytest.fail("tests/c/libmock_rccl.so is not built (run __graft_entry__.build())")
    r = subprocess.run([BIN, str(log_n), str(cols), str(log_lde), str(cap), str(threads), str(log_k)],
                       capture_output=True, text=True, timeout=180, env=dict(os.environ, BJ_TEST_MOCK_RCCL=mock))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "c_caller ok (collective also over RCCL's API" in r.stdout, r.stdout
    # bj_comm_info / bj_comm_check_world through RCCL's API: ncclCommCount = 2, 4, 8 and each
    # rank's ncclCommUserRank; the stand-in's ranks share one GPU and the check must say so
    assert "rccl world check ok at world 2 4 8" in r.stdout, r.stdout
    assert "a failed record rejected on every rank" in r.stdout, r.stdout
    # the link probe bench.py's N > 1 line carries ("link"): one exchange of the commit's own
    # kind and size on every rank, at world 2, 4 and 8 (the mock's rate is a device copy's)
    import re
    links = re.findall(r"^link world (\d+) rank (\d+) kind (\w+) bytes_per_rank (\d+) ms ([\d.]+) gbs_per_rank ([\d.]+)$",
                       r.stdout, re.M)
    for world in (2, 4, 8):
        got = [l for l in links if int(l[0]) == world]
        assert sorted(int(l[1]) for l in got) == list(range(world)), (world, got)
        kind = "all_to_all" if world > (1 << log_lde) else "all_gather"
        block = 8 * (((1 << log_n) << log_k) // world) * (cols // world) * (1 << (log_lde - log_k)) \
            if kind == "all_to_all" else 8 * (1 << log_n) * (cols // world)
        for l in got:
            assert l[2] == kind and int(l[3]) == (world - 1) * block and float(l[4]) > 0, (world, l)


@pytest.mark.gpu
def test_c_caller_release_returns_memory():
    """Commits of three sizes cache tables and workspace; bj_release_tables + bj_release_workspace
    (the Rust BjTables guard's Drop, integration/rust/ffi.rs) give the device memory back."""
    _need_bin()
    r = subprocess.run([BIN, "release"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "c_caller release ok" in r.stdout, r.stdout
