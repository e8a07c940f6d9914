"""Training-loop fixtures produced by the REFERENCE (epfml/powersgd) on CPU.

Run in the dev container only (the reference is not on the GPU box):

    PYTHONPATH=/root/reference python tests/golden/make_golden_training.py

T1 pins the reference's north-star entry point ``optimizer_step`` (powersgd/__init__.py:7-25)
inside the data-parallel flow the paper code uses (one process per worker, gloo, every rank
running the same optimizer, train_pytorch.py:106-131 without the model): per step each rank
accumulates a fresh gradient into ``p.grad`` (autograd's accumulation onto the residual the
previous step left there, README.md:39-42), then calls ``optimizer_step(SGD, PowerSGD)``. The
fixture stores, per step, the parameters after the optimizer step, every rank's ``p.grad``
(the error-feedback residual) and every rank's aggregated gradients.

The same fixture pins the DDP communication hook (powersgd_amd/ddp.py): a DDP model whose
loss is sum_i <p_i, g_i,t> has exactly g_i,t as its local gradient, so the hook + SGD must
reproduce the same parameters and aggregated gradients.

Gradients come from the portable hash generator (powersgd_amd.workloads.hash_tensors), the
initial parameters too; P/Q initial state (the reference's CPU Generator) is stored.
"""
from __future__ import annotations

import json
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
if "/root/reference" not in sys.path:
    sys.path.insert(0, "/root/reference")

from powersgd_amd.workloads import hash_tensors  # noqa: E402

SHAPES = [(20, 3, 3, 3), (20,), (24, 20, 3, 3), (24,), (1, 24), (1,), (64, 32), (48, 64, 1, 1),
          (96, 40), (96, 40)]
# name -> (rank, mcr, iters, start_after, steps, world, lr, momentum, weight_decay)
SCENARIOS = {
    "T1_sgd_r2_i2_w2": (2, 2, 2, 1, 4, 2, 0.05, 0.9, 1e-4),
    "T1_sgd_r1_i1_w1": (1, 2, 1, 1, 4, 1, 0.1, 0.0, 0.0),
    "T1_sgd_r4_i3_w2": (4, 1.5, 3, 0, 3, 2, 0.02, 0.5, 0.0),
}


def init_params():
    return [torch.from_numpy(x.copy()) * 0.1 for x in hash_tensors(SHAPES, seed=3000)]


def step_grads(t, rank_id):
    return [torch.from_numpy(x) for x in hash_tensors(SHAPES, seed=4000 + 10 * t + rank_id)]


def run(name, rank_id=0):
    from powersgd import Config, PowerSGD, optimizer_step

    rank, mcr, iters, start, steps, world, lr, mom, wd = SCENARIOS[name]
    params = [torch.nn.Parameter(p.clone()) for p in init_params()]
    opt = torch.optim.SGD(params, lr=lr, momentum=mom, weight_decay=wd)
    psgd = PowerSGD(params, Config(rank=rank, min_compression_rate=mcr, num_iters_per_step=iters,
                                   start_compressing_after_num_steps=start))
    rec = {"mask": np.array(psgd.is_compressed_mask, dtype=np.bool_),
           "p0": psgd._powersgd._ps_buffer.numpy().copy(),
           "q0": psgd._powersgd._qs_buffer.numpy().copy()}
    captured = {}
    orig_aggregate = psgd.aggregate

    def spy(grads):  # record what optimizer.step() is handed (the aggregated gradients)
        outs = orig_aggregate(grads)
        captured["outs"] = [o.detach().clone() for o in outs]
        return outs

    psgd.aggregate = spy
    for t in range(steps):
        for p, g in zip(params, step_grads(t, rank_id)):
            if p.grad is None:
                p.grad = g.clone()
            else:
                p.grad.add_(g)  # autograd accumulates onto the residual
        optimizer_step(opt, psgd)
        for i, p in enumerate(params):
            rec[f"s{t}_param_{i}"] = p.detach().numpy().copy()
            rec[f"s{t}_grad_{i}"] = p.grad.detach().numpy().copy()
            rec[f"s{t}_avg_{i}"] = captured["outs"][i].numpy().copy()
        rec[f"s{t}_step"] = np.array([psgd.step_counter, psgd._powersgd.step_counter])
    return rec


def _worker(rank_id, world, name, initfile, outdir):
    torch.distributed.init_process_group("gloo", init_method=f"file://{initfile}", rank=rank_id,
                                         world_size=world)
    torch.set_num_threads(1)
    rec = run(name, rank_id)
    np.savez_compressed(os.path.join(outdir, f"r{rank_id}.npz"), **rec)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def main():
    manifest = {"shapes": [list(s) for s in SHAPES], "param_seed": 3000, "param_scale": 0.1,
                "grad_seed": 4000, "scenarios": {}}
    for name, sc in SCENARIOS.items():
        world = sc[5]
        if world == 1:
            merged = {f"rank0_{k}": v for k, v in run(name).items()}
        else:
            with tempfile.TemporaryDirectory() as td:
                torch.multiprocessing.spawn(_worker, args=(world, name, os.path.join(td, "init"), td),
                                            nprocs=world, join=True)
                merged = {}
                for r in range(world):
                    with np.load(os.path.join(td, f"r{r}.npz")) as z:
                        for k in z.files:
                            merged[f"rank{r}_{k}"] = z[k]
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **merged)
        rank, mcr, iters, start, steps, world, lr, mom, wd = sc
        manifest["scenarios"][name] = dict(rank=rank, mcr=mcr, iters=iters, start=start, steps=steps,
                                           world=world, lr=lr, momentum=mom, weight_decay=wd)
        print(name, flush=True)
    with open(os.path.join(HERE, "training_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
