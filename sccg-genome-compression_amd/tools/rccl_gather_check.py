"""RCCL smoke of bench.py's record gather (all_gather_into_tensor of sizes + gather to rank 0) at
whatever world size torchrun gives (the 1-GPU box: world 1).  Prints the gathered sizes."""
import os

import torch
import torch.distributed as dist

dist.init_process_group(backend="nccl")
rank, world = dist.get_rank(), dist.get_world_size()
local = int(os.environ.get("LOCAL_RANK", "0"))
torch.cuda.set_device(local)
dev = torch.device("cuda", local)
d_out = (torch.arange(1 << 20, device=dev) % 251).to(torch.uint8)
n = 1000 + rank
sz = torch.tensor([n], dtype=torch.int64, device=dev)
sizes = torch.empty(world, dtype=torch.int64, device=dev)
dist.all_gather_into_tensor(sizes, sz)
mx = int(sizes.max().item())
parts = [torch.empty(mx, dtype=torch.uint8, device=dev) for _ in range(world)] if rank == 0 else None
dist.gather(d_out[:mx], parts, dst=0)
torch.cuda.synchronize()
if rank == 0:
    ok = all(torch.equal(p[: int(sizes[i])], d_out[: int(sizes[i])]) for i, p in enumerate(parts))
    print("rccl gather ok" if ok else "rccl gather MISMATCH", sizes.tolist())
dist.destroy_process_group()
