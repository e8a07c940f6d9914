"""Diagnose: (7,1000)-style matrices at rank 4, I=2, step 1 vs the oracle, per kernel option."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from oracle import powersgd_oracle as O
from powersgd_amd import Config, PowerSGD
from powersgd_amd.workloads import hash_tensors

DEV = torch.device("cuda:0")
shapes = [tuple(map(int, s.split("x"))) for s in sys.argv[1].split(",")]
rank, iters = int(sys.argv[2]), int(sys.argv[3])
psgd = PowerSGD([torch.zeros(s, device=DEV) for s in shapes], Config(rank, 0.5, iters, 0))
res = [torch.zeros(s) for s in shapes]
for t in range(3):
    ora = O.policy_init([torch.zeros(s) for s in shapes], rank, 0.5, iters, 0)
    ora.codec.p_flat.copy_(psgd._powersgd._ps_buffer.cpu())
    ora.codec.q_flat.copy_(psgd._powersgd._qs_buffer.cpu())
    ora.step = psgd.step_counter
    ora.codec.step = psgd._powersgd.step_counter
    fresh = [torch.from_numpy(f) for f in hash_tensors(shapes, seed=300 + t)]
    inputs = [r + f for r, f in zip(res, fresh)]
    g = [x.to(DEV) for x in inputs]
    gc = [x.clone() for x in inputs]
    o = psgd.aggregate(g)
    oc = O.policy_step(ora, gc)
    torch.cuda.synchronize()
    for i, x in enumerate(inputs):
        eo = float((o[i].cpu() - oc[i]).norm() / x.norm())
        er = float((g[i].cpu() - gc[i]).norm() / x.norm())
        print(f"t={t} i={i} {shapes[i]} out={eo:.2e} res={er:.2e}")
    res = [x.cpu() for x in g]
