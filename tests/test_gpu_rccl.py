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
