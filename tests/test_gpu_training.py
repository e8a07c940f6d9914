"""optimizer_step and the DDP hook on the GPU against the REFERENCE's training-loop fixtures
(tests/golden/make_golden_training.py: reference ``optimizer_step`` + SGD, gloo, world size
1 and 2, four steps with warm-up and error feedback).

* ``powersgd_amd.optimizer_step`` (reference powersgd/__init__.py:7-25): per step the fresh
  gradient is accumulated into ``p.grad`` (which holds the residual), then
  ``optimizer_step(SGD, PowerSGD)``; the parameters, ``p.grad`` (residual) and the averaged
  gradients handed to ``optimizer.step()`` are compared with the reference's.
* ``powersgd_amd.ddp.powersgd_hook``: a DistributedDataParallel model whose loss is
  sum_i <p_i, g_i,t> (so its local gradients are exactly the fixture's g_i,t), SGD, zero_grad
  each step; ``p.grad`` after backward (the hook's result) and the parameters after the step
  are compared with the reference flow. The model is bucketed in small buckets so DDP builds
  several buckets and rebuilds them after the first iteration.

World size 2 runs as two processes on cuda:0 over gloo. Tolerances (free-running, multi-step,
SURVEY §8(c)): averaged gradients and residuals within TOL_FREE of the step's input-gradient
norm; parameters within TOL_FREE of the accumulated update norm.
"""
import os
import tempfile

import numpy as np
import pytest
import torch

from parity_log import check
from training_io import SHAPES, TMAN, init_params, load, step_grads

pytestmark = pytest.mark.gpu
TOL_FREE = 1e-4
DEV = torch.device("cuda:0")


def _rel(a, b, scale) -> float:
    a = a.detach().double().cpu()
    b = torch.as_tensor(b).double()
    return float((a - b).norm()) / max(float(torch.as_tensor(scale).double().norm()), 1e-30)


def _inject(psgd, want):
    psgd._powersgd._ps_buffer.copy_(torch.from_numpy(want["rank0_p0"]).to(DEV))
    psgd._powersgd._qs_buffer.copy_(torch.from_numpy(want["rank0_q0"]).to(DEV))


def _optimizer_step_run(name, rank_id, world):
    from powersgd_amd import Config, PowerSGD, optimizer_step

    sc = TMAN["scenarios"][name]
    want = load(name)
    p_init = init_params()
    params = [torch.nn.Parameter(p.clone().to(DEV)) for p in p_init]
    opt = torch.optim.SGD(params, lr=sc["lr"], momentum=sc["momentum"], weight_decay=sc["weight_decay"])
    psgd = PowerSGD(params, Config(sc["rank"], sc["mcr"], sc["iters"], sc["start"]))
    assert psgd.is_compressed_mask == list(want[f"rank{rank_id}_mask"])
    _inject(psgd, want)
    seen = {}
    orig = psgd.aggregate

    def spy(grads):
        seen["in"] = [g.detach().cpu().clone() for g in grads]
        seen["out"] = orig(grads)
        return seen["out"]

    psgd.aggregate = spy
    for t in range(sc["steps"]):
        for p, g in zip(params, step_grads(t, rank_id)):
            if p.grad is None:
                p.grad = g.clone().to(DEV)
            else:
                p.grad.add_(g.to(DEV))  # autograd accumulates onto the residual
        optimizer_step(opt, psgd)
        torch.cuda.synchronize()
        pre = f"rank{rank_id}_s{t}_"
        for i, p in enumerate(params):
            g = seen["in"][i]
            check(_rel(seen["out"][i], want[pre + f"avg_{i}"], g), TOL_FREE, name, rank_id, t, i, "avg")
            check(_rel(p.grad, want[pre + f"grad_{i}"], g), TOL_FREE, name, rank_id, t, i, "residual")
            check(_rel(p, want[pre + f"param_{i}"], torch.from_numpy(want[pre + f"param_{i}"]) - p_init[i]),
                  TOL_FREE, name, rank_id, t, i, "param")
        assert [psgd.step_counter, psgd._powersgd.step_counter] == list(want[pre + "step"])


class _Probe(torch.nn.Module):
    """loss = sum_i <p_i, c_i>: the local gradient of p_i is exactly c_i."""

    def __init__(self, init):
        super().__init__()
        self.ps = torch.nn.ParameterList([torch.nn.Parameter(p.clone()) for p in init])

    def forward(self, cs):
        return sum((p * c).sum() for p, c in zip(self.ps, cs))


def _ddp_run(name, rank_id, world):
    from torch.nn.parallel import DistributedDataParallel as DDP

    from powersgd_amd import Config
    from powersgd_amd.ddp import PowerSGDState, powersgd_hook

    sc = TMAN["scenarios"][name]
    want = load(name)
    p_init = init_params()
    model = _Probe(p_init).to(DEV)
    params = list(model.parameters())
    opt = torch.optim.SGD(params, lr=sc["lr"], momentum=sc["momentum"], weight_decay=sc["weight_decay"])
    # ~10 KB buckets: several buckets, reverse-order bucketing, rebuilt after iteration 1
    ddp = DDP(model, device_ids=[0], bucket_cap_mb=0.01)
    state = PowerSGDState(Config(sc["rank"], sc["mcr"], sc["iters"], sc["start"]), params=params)
    _inject(state.powersgd, want)
    ddp.register_comm_hook(state, powersgd_hook)
    resid = [torch.zeros(s) for s in SHAPES]
    for t in range(sc["steps"]):
        cs = [g.to(DEV) for g in step_grads(t, rank_id)]
        ddp(cs).backward()
        torch.cuda.synchronize()
        pre = f"rank{rank_id}_s{t}_"
        ins = [r + g for r, g in zip(resid, step_grads(t, rank_id))]  # the reference's p.grad
        for i, p in enumerate(params):
            check(_rel(p.grad, want[pre + f"avg_{i}"], ins[i]), TOL_FREE, name, rank_id, t, i, "ddp-avg")
        opt.step()
        opt.zero_grad()
        torch.cuda.synchronize()
        for i, p in enumerate(params):
            check(_rel(state.views[i], want[pre + f"grad_{i}"], ins[i]), TOL_FREE, name, rank_id, t, i,
                  "ddp-residual")
            check(_rel(p, want[pre + f"param_{i}"], torch.from_numpy(want[pre + f"param_{i}"]) - p_init[i]),
                  TOL_FREE, name, rank_id, t, i, "ddp-param")
        resid = [torch.from_numpy(want[pre + f"grad_{i}"]) for i in range(len(SHAPES))]
    assert [state.powersgd.step_counter, state.powersgd._powersgd.step_counter] == \
        list(want[f"rank{rank_id}_s{sc['steps'] - 1}_step"])


def _worker(rank_id, world, name, initfile, which):
    torch.distributed.init_process_group("gloo", init_method=f"file://{initfile}", rank=rank_id, world_size=world)
    try:
        (_ddp_run if which == "ddp" else _optimizer_step_run)(name, rank_id, world)
        torch.distributed.barrier()
    finally:
        torch.distributed.destroy_process_group()


def _spawn(name, which):
    world = TMAN["scenarios"][name]["world"]
    with tempfile.TemporaryDirectory() as td:
        torch.multiprocessing.spawn(_worker, args=(world, name, os.path.join(td, "init"), which), nprocs=world,
                                    join=True)


@pytest.mark.parametrize("name", sorted(TMAN["scenarios"]))
def test_optimizer_step_matches_reference(name):
    if TMAN["scenarios"][name]["world"] == 1:
        _optimizer_step_run(name, 0, 1)  # no process group: the reference's single-process path
    else:
        _spawn(name, "opt")


@pytest.mark.parametrize("name", sorted(TMAN["scenarios"]))
def test_ddp_hook_matches_reference(name):
    _spawn(name, "ddp")


def test_optimizer_step_keeps_held_outputs():
    """outputs handed out by one step (p.grad = out, or saved elsewhere) are never
    overwritten by the next step (the reference returns fresh tensors, :153)."""
    from powersgd_amd import Config, PowerSGD

    shapes = [(64, 32), (64, 32), (16,)]
    psgd = PowerSGD([torch.zeros(s, device=DEV) for s in shapes], Config(1, 2, 2, 0))
    g1 = [torch.randn(s, device=DEV) for s in shapes]
    out1 = psgd.aggregate(g1)
    keep = [o.clone() for o in out1]
    g2 = [torch.randn(s, device=DEV) for s in shapes]
    out2 = psgd.aggregate(g2)
    torch.cuda.synchronize()
    for a, b in zip(out1, keep):
        assert torch.equal(a, b)
    assert all(a.data_ptr() != b.data_ptr() for a, b in zip(out1, out2))


def test_fresh_gradient_tensors_every_step_no_host_sync():
    """zero_grad(set_to_none=True) style: brand-new gradient tensors each step. The pointer
    tables are selected/uploaded stream-ordered (no host synchronisation); results must equal
    a run that reuses one set of tensors."""
    from powersgd_amd import Config, PowerSGD

    shapes = [(96, 40), (96, 40), (64, 32, 3, 3), (7,)]
    a = PowerSGD([torch.zeros(s, device=DEV) for s in shapes], Config(2, 2, 2, 0))
    b = PowerSGD([torch.zeros(s, device=DEV) for s in shapes], Config(2, 2, 2, 0))
    ga = [torch.zeros(s, device=DEV) for s in shapes]
    for t in range(8):
        fresh = [torch.randn(s, generator=torch.Generator().manual_seed(t * 10 + i)) for i, s in enumerate(shapes)]
        for x, f in zip(ga, fresh):
            x.add_(f.to(DEV))
        gb = [x.clone() for x in ga]  # new allocations every step (6+ distinct pointer sets)
        oa = a.aggregate(ga)
        ob = b.aggregate(gb)
        torch.cuda.synchronize()
        for x, y in zip(oa + ga, ob + gb):
            assert torch.equal(x, y), t
        del gb
