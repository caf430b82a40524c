"""Probe: can two ranks share one GPU under RCCL (torch.distributed 'nccl')?  Prints one line per rank."""
import os
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"]); world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda:0"))
x = torch.full((4,), float(rank), device="cuda:0")
out = [torch.empty_like(x) for _ in range(world)]
dist.all_gather(out, x)
torch.cuda.synchronize()
print(f"rank {rank}: allgather ok {[o[0].item() for o in out]}", flush=True)
dist.destroy_process_group()
