"""The DDP comm hook on a bf16 model against the CPU oracle (the T1
fixtures of tests/test_gpu_training.py cover fp32 models only, and tests/test_gpu_ddp_large.py
checks a size-independent property).

W = 2 processes on cuda:0 over gloo, a bf16 model whose loss is sum_i <p_i, c_i> (so each
rank's local gradient is exactly its c_i), DDP with small buckets (several buckets, rebuilt
after the first iteration), ``powersgd_hook``. Per step every rank records the exact bf16
inputs of its codec (the state's residual after the bucket adds: what the reference's
``p.grad`` holds before ``aggregate``), the ranks all-gather them, and W oracle workers
(oracle/multiworker.py: the reference's aggregate at world size W, threads meeting at its SUM
all-reduce, powersgd.py:172-219) run on exactly those values upcast to fp32 (the reference
raises on bf16 at its bmm). The hook's averages (p.grad after backward) and residuals (bf16)
must match within 4e-3 of the input norm: the bf16 storage bound of SURVEY §8(c) (one bf16
rounding of each stored element, ~2^-9 relative)."""
import os
import tempfile

import pytest
import torch

from parity_log import check
from training_io import SHAPES, init_params, step_grads

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL_BF16 = 4e-3
STEPS = 3


class _Probe(torch.nn.Module):
    def __init__(self, init):
        super().__init__()
        self.ps = torch.nn.ParameterList([torch.nn.Parameter(p.clone()) for p in init])

    def forward(self, cs):
        return sum((p * c).sum() for p, c in zip(self.ps, cs))


def _rel(a, b, scale) -> float:
    return float((a.detach().double().cpu() - b.double()).norm()) / max(float(scale.double().norm()), 1e-30)


def _run(rank_id, world, rank, iters):
    from torch.nn.parallel import DistributedDataParallel as DDP

    from oracle import multiworker as MW
    from oracle import powersgd_oracle as O
    from powersgd_amd import Config
    from powersgd_amd.ddp import PowerSGDState, powersgd_hook

    model = _Probe([p.to(torch.bfloat16) for p in init_params()]).to(DEV)
    params = list(model.parameters())
    ddp = DDP(model, device_ids=[0], bucket_cap_mb=0.01)
    state = PowerSGDState(Config(rank, 2, iters, 0), params=params)
    ddp.register_comm_hook(state, powersgd_hook)
    codec = state.powersgd
    oracles = []
    for _ in range(world):  # every worker starts from this codec's P/Q (the reference's seed-0 init)
        st = O.policy_init([torch.zeros(s) for s in SHAPES], rank, 2, iters, 0)
        st.codec.p_flat.copy_(codec._powersgd._ps_buffer.cpu())
        st.codec.q_flat.copy_(codec._powersgd._qs_buffer.cpu())
        oracles.append(st)
    seen = {}
    orig = codec.aggregate

    def spy(grads):
        seen["in"] = [g.detach().float().cpu() for g in grads]  # the exact bf16 inputs, upcast
        return orig(grads)

    codec.aggregate = spy
    for t in range(STEPS):
        cs = [g.to(DEV, torch.bfloat16) for g in step_grads(t, rank_id)]
        ddp(cs).backward()
        torch.cuda.synchronize()
        ins = [None] * world
        torch.distributed.all_gather_object(ins, seen["in"])
        gc = [[x.clone() for x in ins[w]] for w in range(world)]
        want = MW.run_workers(oracles, gc)
        for i, p in enumerate(params):
            # the average mixes every rank's input: measured against the largest of them
            scale = max((ins[w][i] for w in range(world)), key=lambda x: float(x.norm()))
            check(_rel(p.grad, want[rank_id][i], scale), TOL_BF16, rank, iters, rank_id, t, i, "ddp-bf16-avg")
            check(_rel(state.views[i], gc[rank_id][i], scale), TOL_BF16, rank, iters, rank_id, t, i,
                  "ddp-bf16-residual")
        for p in params:
            p.grad = None


def _worker(rank_id, world, initfile, rank, iters):
    torch.distributed.init_process_group("gloo", init_method=f"file://{initfile}", rank=rank_id, world_size=world)
    try:
        _run(rank_id, world, rank, iters)
        torch.distributed.barrier()
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.parametrize("rank,iters", [(2, 2), (1, 1), (4, 3)])
def test_ddp_hook_bf16_matches_oracle(rank, iters):
    with tempfile.TemporaryDirectory() as td:
        torch.multiprocessing.spawn(_worker, args=(2, os.path.join(td, "init"), rank, iters), nprocs=2, join=True)
