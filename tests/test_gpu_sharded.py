"""GPU parity of the coset-sharded LDE (bj_lde_coeffs_d / bj_lde_shard_d) and of the
multi-process sharded commit on one card: the native collective (bj_sharded_commit_d) in G
processes joined by a gloo group through the callback transport (RCCL needs one GPU per rank).

Each shard's LDE must equal the matching leaf range of the oracle's full LDE, bit for bit,
for G <= D (whole cosets), G > D (folded sub-cosets, F = G/D up to 8) and sizes on both the
generic and the register-resident (n >= 2^18) NTT paths."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_mod():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    import boojum_amd
    boojum_amd.load()
    return torch


@pytest.mark.parametrize("c,log_n,log_d,log_g", [
    (3, 6, 1, 1), (3, 6, 1, 2), (2, 8, 2, 1), (2, 8, 2, 3), (5, 10, 1, 4), (2, 12, 3, 3), (2, 12, 1, 3),
    (1, 19, 1, 2), (1, 19, 2, 3), (1, 18, 1, 1)])
def test_lde_shard_matches_full_lde(torch_mod, c, log_n, log_d, log_g):
    torch = torch_mod
    from boojum_amd._lib import call
    from boojum_amd.field import stream_of, to_device, to_host
    n, nl = 1 << log_n, 1 << (log_n + log_d)
    m = nl >> log_g
    x = np.random.default_rng(c * 1000 + log_n * 10 + log_g).integers(0, O.P, size=(c, n), dtype=np.uint64)
    _, ref = O.lde(x, log_d, threads=8)
    ref = ref.reshape(c, nl)
    tr = to_device(x)
    co = torch.empty((c, n), dtype=torch.int64, device="cuda")
    call("bj_lde_coeffs_d", tr.data_ptr(), c, n, log_n, co.data_ptr(), n, stream_of(co))
    work = torch.empty((c, m), dtype=torch.int64, device="cuda")
    for P in range(1 << log_g):
        lde = torch.empty((c, m), dtype=torch.int64, device="cuda")
        call("bj_lde_shard_d", co.data_ptr(), c, n, log_n, log_d, log_g, P, work.data_ptr(), lde.data_ptr(),
             stream_of(lde))
        got = to_host(lde)
        assert np.array_equal(got, ref[:, P * m:(P + 1) * m]), "shard %d of %d" % (P, 1 << log_g)


@pytest.mark.parametrize("c,log_n,log_d,log_g", [
    (3, 6, 1, 2), (2, 8, 2, 3), (5, 10, 1, 4), (2, 12, 1, 3), (2, 10, 1, 5), (1, 19, 2, 3), (2, 18, 1, 2),
    (1, 20, 1, 4)])
def test_fold_on_sender_matches_full_lde(torch_mod, c, log_n, log_d, log_g):
    """bj_lde_fold_shards_d (every target folded from one read) + bj_lde_shard_folded_d = the
    leaf ranges of the full LDE, for fold factors 2..16 (the fused kernel for F <= 8, the
    per-target fallback above)."""
    torch = torch_mod
    from boojum_amd._lib import call
    from boojum_amd.field import stream_of, to_device, to_host
    n, nl = 1 << log_n, 1 << (log_n + log_d)
    G = 1 << log_g
    m = nl >> log_g
    x = np.random.default_rng(c * 7 + log_n * 3 + log_g).integers(0, O.P, size=(c, n), dtype=np.uint64)
    _, ref = O.lde(x, log_d, threads=8)
    ref = ref.reshape(c, nl)
    tr = to_device(x)
    co = torch.empty((c, n), dtype=torch.int64, device="cuda")
    call("bj_lde_coeffs_d", tr.data_ptr(), c, n, log_n, co.data_ptr(), n, stream_of(co))
    send = torch.full((G, c, m), -1, dtype=torch.int64, device="cuda")
    call("bj_lde_fold_shards_d", co.data_ptr(), c, n, log_n, log_d, log_g, send.data_ptr(), c * m, stream_of(send))
    for P in range(G):
        lde = torch.empty((c, m), dtype=torch.int64, device="cuda")
        call("bj_lde_shard_folded_d", send[P].data_ptr(), c, m, log_n, log_d, log_g, P, lde.data_ptr(),
             stream_of(lde))
        assert np.array_equal(to_host(lde), ref[:, P * m:(P + 1) * m]), "shard %d of %d" % (P, G)


def test_lde_shard_errors(torch_mod):
    from boojum_amd import BoojumError
    from boojum_amd._lib import call
    with pytest.raises(BoojumError):
        call("bj_lde_shard_d", None, 1, 16, 4, 1, 2, 4, None, None, None)   # shard >= G
    with pytest.raises(BoojumError):
        call("bj_lde_shard_d", None, 1, 16, 4, 1, 2, 1, None, None, None)   # G > D without work
    with pytest.raises(BoojumError):
        call("bj_lde_fold_shards_d", None, 1, 16, 4, 1, 1, None, 8, None)    # G == D: nothing to fold
    with pytest.raises(BoojumError):
        call("bj_lde_fold_shards_d", None, 1, 16, 4, 1, 2, None, 7, None)    # shard stride < n_cols * m
    with pytest.raises(BoojumError):
        call("bj_lde_shard_folded_d", None, 1, 8, 4, 1, 2, 4, None, None)    # shard >= G


@pytest.mark.parametrize("world,cfg", [(2, (8, 10, 1, 16)), (4, (8, 9, 1, 2)), (2, (48, 10, 2, 16)),
                                       (4, (64, 12, 1, 4)), (8, (64, 9, 1, 16)), (2, (256, 9, 1, 16)),
                                       (8, (128, 14, 2, 16)),
                                       (4, (64, 12, 1, 4, 0, None, "blake2s")),
                                       (2, (32, 10, 1, 16, 0, None, "keccak256")),
                                       (4, (32, 12, 3, 32, 0, None, None, 1)),     # D = 8, k = 2, cap 32
                                       (8, (32, 12, 2, 16, 0, None, None, 0))])    # D = 4, k = 1, G > D
def test_sharded_commit_multiprocess_one_gpu(torch_mod, world, cfg, tmp_path):
    from sharded_check import run_and_check
    run_and_check(world, cfg, tmp_path, "cuda")
