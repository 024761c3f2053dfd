"""Can two ranks share one GPU under RCCL on this box?  (rehearsal feasibility probe)"""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.full((1024,), float(rank), device="cuda:0")
g = [torch.empty_like(x) for _ in range(world)] if rank == 0 else None
w = dist.gather(x, g, dst=0, async_op=True)
w.wait()
torch.cuda.synchronize()
if rank == 0:
    print("gather ok", [float(t[0]) for t in g])
dist.destroy_process_group()
