"""Even product in isolation on cold gradients: psgd_compress(step 0, it 0) over S rotating
gradient sets (orth P + even product + reduce, no final pass between them), to separate the
product's own cold rate from interference with the previous step's final-pass writes.
usage: python tools/exp_even.py [config] [mode: even|step]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from powersgd_amd import Config, PowerSGD  # noqa: E402
from powersgd_amd.workloads import CONFIGS  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3_resnet50_r4"
mode = sys.argv[2] if len(sys.argv) > 2 else "even"
if "x" in cfg:  # "NxM[,NxM...]:rank"
    sh, rk = cfg.split(":")
    c = dict(shapes=[tuple(int(v) for v in t.split("x")) for t in sh.split(",")], rank=int(rk), iters=2, mcr=1.0)
else:
    c = CONFIGS[cfg]
dev = torch.device("cuda:0")
S = 4
gen = torch.Generator(device=dev).manual_seed(1)
sets = [[torch.randn(s, generator=gen, device=dev) for s in c["shapes"]] for _ in range(S)]
psgd = PowerSGD([torch.zeros(s, device=dev) for s in c["shapes"]], Config(c["rank"], c["mcr"], c["iters"], 0))
cb = psgd._powersgd
stream = torch.cuda.current_stream().cuda_stream
comps = [[g for g, m in zip(sets[k], psgd.is_compressed_mask) if m] for k in range(S)]
outs = [torch.empty(cb._out_numel, device=dev) for _ in range(S)]
for t in range(60):
    k = t % S
    cb._table.fill(comps[k])
    ptrs = cb._table.comp_addr()
    cb._plan.compress(ptrs, 0, 0, stream)
    if mode == "step":  # then the apply pass over the same set (residual + output writes)
        cb._plan.decompress(ptrs, outs[k].data_ptr(), 0, 1, stream)
torch.cuda.synchronize()
print("done", cfg, mode)
