import os, sys, datetime, torch, torch.distributed as dist
rank = int(os.environ["RANK"]); world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", init_method="file://" + sys.argv[1], rank=rank, world_size=world,
                        timeout=datetime.timedelta(seconds=60), device_id=torch.device("cuda", 0))
x = torch.full((4,), rank + 1, device="cuda", dtype=torch.int64)
out = torch.empty(4 * world, device="cuda", dtype=torch.int64)
dist.all_gather_into_tensor(out, x)
torch.cuda.synchronize()
print("rank", rank, out.tolist(), flush=True)
dist.destroy_process_group()
