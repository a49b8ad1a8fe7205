"""Can RCCL run several ranks on ONE GPU (the gpurun box has one)?  Each rank all-gathers a
small tensor over backend 'nccl' on cuda:0 and checks the result.
Usage: torchrun --nproc-per-node 2 --master-addr 127.0.0.1 tools/rccl_probe.py"""
import datetime
import os

import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev, timeout=datetime.timedelta(seconds=60))
x = torch.full((4,), float(rank), device=dev)
out = torch.empty(4 * world, device=dev)
dist.all_gather_into_tensor(out, x)
torch.cuda.synchronize()
want = torch.arange(world, dtype=torch.float32, device=dev).repeat_interleave(4)
print(f"rank {rank}: all_gather ok={bool(torch.equal(out, want))} {out.tolist()}", flush=True)
dist.destroy_process_group()
