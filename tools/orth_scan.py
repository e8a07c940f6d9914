"""Scan the orthonormalisation kernel's duration vs panel rows k and number of units
(run under rocprofv3 --kernel-trace --stats)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from powersgd_amd import Config, PowerSGD

dev = torch.device("cuda:0")
cases = [((2048, 64), 54, 4), ((2048, 64), 1, 4), ((256, 64), 54, 4), ((8192, 64), 54, 4),
         ((2048, 64), 54, 1), ((2048, 64), 54, 2)]
for shape, count, rank in cases:
    shapes = [shape] * count
    grads = [torch.randn(s, device=dev) for s in shapes]
    p = PowerSGD([torch.zeros(s, device=dev) for s in shapes], Config(rank, 0.1, 1, 0))
    for _ in range(20):
        p.aggregate(grads)
    torch.cuda.synchronize()
    torch.cuda.nvtx.range_push if False else None
    print("case", shape, count, rank, flush=True)
