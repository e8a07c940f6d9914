"""Pin the oracle's optimizer_step (oracle/powersgd_oracle.py) bitwise against the reference's
training-loop fixtures (tests/golden/make_golden_training.py, reference powersgd/__init__.py:7-25):
SGD + PowerSGD over gloo at world size 1 and 2."""
import os
import tempfile

import numpy as np
import pytest
import torch

from oracle import powersgd_oracle as O
from training_io import TMAN, init_params, load, step_grads


def _run(name, rank_id=0, world=1, allreduce=None):
    sc = TMAN["scenarios"][name]
    params = [torch.nn.Parameter(p.clone()) for p in init_params()]
    opt = torch.optim.SGD(params, lr=sc["lr"], momentum=sc["momentum"], weight_decay=sc["weight_decay"])
    ps = O.policy_init(params, sc["rank"], sc["mcr"], sc["iters"], sc["start"])
    rec = {"mask": np.array(ps.mask), "p0": ps.codec.p_flat.numpy().copy(), "q0": ps.codec.q_flat.numpy().copy()}
    for t in range(sc["steps"]):
        for p, g in zip(params, step_grads(t, rank_id)):
            if p.grad is None:
                p.grad = g.clone()
            else:
                p.grad.add_(g)
        avg = O.optimizer_step(opt, ps, params, world, allreduce)
        for i, p in enumerate(params):
            rec[f"s{t}_param_{i}"] = p.detach().numpy().copy()
            rec[f"s{t}_grad_{i}"] = p.grad.detach().numpy().copy()
            rec[f"s{t}_avg_{i}"] = avg[i].detach().numpy().copy()
        rec[f"s{t}_step"] = np.array([ps.step, ps.codec.step])
    return {f"rank{rank_id}_{k}": v for k, v in rec.items()}


def _same(got, want):
    for k, v in want.items():
        assert k in got, k
        assert np.array_equal(got[k], v), (k, float(np.max(np.abs(got[k].astype(np.float64) - v))))


def _worker(rank_id, world, name, initfile, outdir):
    torch.distributed.init_process_group("gloo", init_method=f"file://{initfile}", rank=rank_id, world_size=world)
    torch.set_num_threads(1)
    rec = _run(name, rank_id, world, lambda b: torch.distributed.all_reduce(b))
    np.savez(os.path.join(outdir, f"r{rank_id}.npz"), **rec)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("name", sorted(TMAN["scenarios"]))
def test_oracle_optimizer_step_bitwise(name):
    world = TMAN["scenarios"][name]["world"]
    want = load(name)
    if world == 1:
        _same(_run(name), want)
        return
    with tempfile.TemporaryDirectory() as td:
        torch.multiprocessing.spawn(_worker, args=(world, name, os.path.join(td, "init"), td), nprocs=world, join=True)
        got = {}
        for r in range(world):
            with np.load(os.path.join(td, f"r{r}.npz")) as z:
                got.update({k: z[k] for k in z.files})
    _same(got, want)
