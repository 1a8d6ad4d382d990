"""The bench's N > 1 communicator path on the one GPU of the box: a torch.distributed "nccl"
(RCCL) process group of one rank with the bench's options (high-priority stream), and
NativeComm.rccl over it (rank 0 makes the RCCL unique id, the group broadcasts it,
ncclCommInitRank) driving bj_sharded_commit_d.  A one-rank group cannot show bandwidth or
overlap; it checks that the calls the 8-GPU run depends on are accepted by this torch/RCCL
build and give the one-GPU commit."""

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg(tmp_path_factory):
    import torch
    import torch.distributed as dist
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    torch.cuda.set_device(0)
    store = dist.FileStore(str(tmp_path_factory.mktemp("rccl") / "store"), 1)
    opts = dist.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=torch.device("cuda", 0),
                            pg_options=opts)
    yield torch
    dist.destroy_process_group()


@pytest.mark.parametrize("log_lde,log_k", [(2, 2), (3, 1)])
def test_native_commit_over_process_group_comm(pg, log_lde, log_k):
    torch = pg
    from boojum_amd import commit
    from boojum_amd.sharded import NativeComm, native_sharded_commit
    n_cols, log_n, cap = 16, 13, 16
    comm = NativeComm.rccl()
    try:
        trace = commit.synthetic_trace(n_cols, log_n)
        r = native_sharded_commit(comm, trace, n_cols, log_n, log_lde, cap, log_commit_cosets=log_k)
        ws = commit.witness_commit(trace, 1 << log_lde, cap, fri_lde_factor=1 << log_k)
        torch.cuda.synchronize()
        nd = (1 << log_n) << log_lde
        assert torch.equal(r.lde.permute(1, 0, 2).reshape(n_cols, nd), ws.lde.view(n_cols, nd))
        assert torch.equal(r.leaves, ws.leaves) and torch.equal(r.nodes, ws.nodes) and torch.equal(r.cap, ws.cap)
    finally:
        comm.close()


def _exchange(comm, kind, send, recv, nbytes):
    from boojum_amd._lib import call
    from boojum_amd.field import stream_of
    call("bj_comm_exchange_d", comm.handle, kind, send.data_ptr(), recv.data_ptr(), nbytes, stream_of(recv))


@pytest.mark.parametrize("make", ["world1", "process_group"])
def test_rccl_exchange_calls(pg, make):
    """bj_comm_exchange_d over a one-rank RCCL communicator issues the real RCCL calls the N > 1
    commit makes (ncclAllGather, in place and not; grouped ncclSend / ncclRecv for the
    all-to-all), which the commit itself skips at world 1: the bytes must arrive unchanged."""
    torch = pg
    from boojum_amd.sharded import XCHG_ALL_GATHER, XCHG_ALL_TO_ALL, NativeComm
    comm = NativeComm.rccl_world1() if make == "world1" else NativeComm.rccl()
    try:
        g = torch.Generator(device="cuda").manual_seed(7)
        for n in (1, 1000, 1 << 20):
            src = torch.randint(-2**62, 2**62, (n,), dtype=torch.int64, device="cuda", generator=g)
            for kind in (XCHG_ALL_GATHER, XCHG_ALL_TO_ALL):
                dst = torch.zeros_like(src)
                _exchange(comm, kind, src, dst, 8 * n)
                torch.cuda.synchronize()
                assert torch.equal(dst, src)
            inplace = src.clone()
            _exchange(comm, XCHG_ALL_GATHER, inplace, inplace, 8 * n)
            torch.cuda.synchronize()
            assert torch.equal(inplace, src)
    finally:
        comm.close()


def test_exchange_rejects_bad_arguments(pg):
    torch = pg
    from boojum_amd._lib import BoojumError
    from boojum_amd.sharded import NativeComm
    comm = NativeComm.rccl_world1()
    try:
        a = torch.zeros(4, dtype=torch.int64, device="cuda")
        with pytest.raises(BoojumError):
            _exchange(comm, 7, a, a, 32)
        with pytest.raises(BoojumError):
            _exchange(comm, 0, a, a, 12)
    finally:
        comm.close()


@pytest.mark.parametrize("make", ["world1", "process_group"])
def test_rccl_comm_info_and_world_check(pg, make):
    """bj_comm_info on the real RCCL: ncclCommCount 1, ncclCommUserRank 0, ncclCommCuDevice the
    current device (torch's), its PCI bus id; bj_comm_check_world accepts the one-rank world.
    The N > 1 bench line carries every rank's record from the same call."""
    torch = pg
    from boojum_amd.sharded import NativeComm
    comm = NativeComm.rccl_world1() if make == "world1" else NativeComm.rccl()
    try:
        info = comm.info()
        assert info["kind"] == "rccl"
        assert (info["world"], info["rank"], info["transport_count"], info["transport_rank"]) == (1, 0, 1, 0)
        assert info["device"] == torch.cuda.current_device()
        assert info["pci_bus_id"] and info["host"]
        ok, infos, msg = comm.check_world(torch.cuda.current_stream().cuda_stream)
        assert ok, msg
        assert infos == [info]
    finally:
        comm.close()
