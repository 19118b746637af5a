"""Can two ranks share one GPU under RCCL on this image?  (a probe for exercising the engine's N > 1
data-parallel path on a one-GPU box: torch.distributed.run --nproc-per-node 2, both ranks on cuda:0)."""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.full((4,), float(rank + 1), device="cuda:0")
dist.all_reduce(x)
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce -> {x.tolist()}", flush=True)
dist.destroy_process_group()
