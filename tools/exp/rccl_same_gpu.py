"""Probe: can two ranks share one GPU with the RCCL backend (send/recv + all_reduce)?"""
import os
import torch
import torch.distributed as dist

dist.init_process_group("nccl")
r = dist.get_rank()
torch.cuda.set_device(0)
t = torch.full((4,), float(r + 1), device="cuda:0")
dist.all_reduce(t)
u = torch.zeros(4, device="cuda:0")
if r == 0:
    dist.send(t * 10, 1)
else:
    dist.recv(u, 0)
torch.cuda.synchronize()
print(f"rank {r}: allreduce {t.tolist()} recv {u.tolist()}", flush=True)
dist.destroy_process_group()
