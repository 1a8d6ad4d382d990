"""The RCCL (backend "nccl") calls of the sharded commit, on a one-rank group on the one GPU of
the box: the in-place all-gather and the all-to-all of boojum_amd/sharded.py with async handles
ordering the compute stream, under the bench's process-group options (high-priority stream).
A one-rank group cannot show bandwidth or overlap; it checks that the calls, options and
stream ordering the 8-GPU run depends on are accepted by this torch/RCCL build."""

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


def test_all_gather_in_place_and_all_to_all(pg):
    torch = pg
    from boojum_amd import sharded
    buf = torch.arange(64, dtype=torch.int64, device="cuda").reshape(8, 8)
    src = buf[2:4].clone()
    h = sharded._all_gather(buf[2:4], buf[2:4], async_op=True)   # in place, one rank
    h.wait()
    assert torch.equal(buf[2:4], src)
    out = torch.empty((4, 8), dtype=torch.int64, device="cuda")
    inp = torch.arange(32, dtype=torch.int64, device="cuda").reshape(4, 8) * 3
    h = sharded._all_to_all(out, inp, async_op=True)
    h.wait()
    y = out + 1                     # ordered after the collective on the current stream
    torch.cuda.synchronize()
    assert torch.equal(y, inp + 1)


def test_cap_all_gather_sync(pg):
    torch = pg
    from boojum_amd import sharded
    cap = torch.empty((4, 4), dtype=torch.int64, device="cuda")
    local = torch.arange(16, dtype=torch.int64, device="cuda").reshape(4, 4)
    sharded._all_gather(cap, local)
    torch.cuda.synchronize()
    assert torch.equal(cap, local)
