"""Tiny torchrun payload for the launcher tests: one gloo all-reduce of rank + 1."""
import os

import torch
import torch.distributed as dist

dist.init_process_group("gloo")
t = torch.tensor([float(dist.get_rank() + 1)])
dist.all_reduce(t)
print(f"allreduce_probe rank {dist.get_rank()} port {os.environ['MASTER_PORT']} {t.item()}",
      flush=True)
dist.destroy_process_group()
