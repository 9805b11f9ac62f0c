"""Probe: can two RCCL ranks share the one GPU of a gpurun box?  (torch.distributed.run
--nproc-per-node 2; both ranks on cuda:0).  Prints the all-reduce result per rank."""
import os
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
x = torch.tensor([rank + 1.0], device=dev)
dist.all_reduce(x, op=dist.ReduceOp.MAX)
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce MAX = {x.item()}", flush=True)
g = torch.cuda.CUDAGraph()
y = torch.zeros(1, device=dev)
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    y.fill_(rank + 1.0)
    dist.all_reduce(y, op=dist.ReduceOp.MAX)
torch.cuda.synchronize()
with torch.cuda.graph(g):
    y.fill_(rank + 1.0)
    dist.all_reduce(y, op=dist.ReduceOp.MAX)
g.replay()
torch.cuda.synchronize()
print(f"rank {rank}: captured all_reduce MAX = {y.item()}", flush=True)
dist.destroy_process_group()
