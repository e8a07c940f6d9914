"""Orthonormalisation kernel timing vs panel count and length (run under rocprofv3)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from powersgd_amd import Config, PowerSGD
DEV = torch.device("cuda:0")
for shapes in ([(4608, 96)], [(96, 4608)] * 1, [(96, 4608)] * 16, [(4096, 64)] * 54, [(64, 64)] * 54):
    psgd = PowerSGD([torch.zeros(s, device=DEV) for s in shapes], Config(4, 0.1, 1, 0))
    g = [torch.randn(s, device=DEV) for s in shapes]
    for _ in range(20):
        psgd.aggregate(g)
    torch.cuda.synchronize()
    torch.cuda.nvtx.range_push("x") if False else None
print("done")
