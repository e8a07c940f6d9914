"""DDP communication hook (powersgd_amd/ddp.py): two processes on cuda:0 with gloo.

DistributedDataParallel + powersgd_hook must hand the optimizer the same averaged gradients
as the reference flow (``PowerSGD.aggregate`` on each rank's local gradients, residual kept as
the next step's starting gradient) applied to the same bucket: a replica model without DDP
runs that flow with this package's PowerSGD and is compared step by step (1e-5 relative:
the two paths differ only in gloo vs in-hook summation order)."""
import os
import tempfile

import pytest
import torch

pytestmark = pytest.mark.gpu


def _worker(rank, world, initfile):
    import torch.distributed as dist
    from torch.nn.parallel import DistributedDataParallel as DDP

    from powersgd_amd import Config, PowerSGD
    from powersgd_amd.ddp import PowerSGDState, powersgd_hook

    dist.init_process_group("gloo", init_method=f"file://{initfile}", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.ReLU(), torch.nn.Linear(128, 96),
                                    torch.nn.ReLU(), torch.nn.Linear(96, 10)).to(dev)
        ref = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.ReLU(), torch.nn.Linear(128, 96),
                                  torch.nn.ReLU(), torch.nn.Linear(96, 10)).to(dev)
        ref.load_state_dict(model.state_dict())
        cfg = Config(rank=2, min_compression_rate=2, num_iters_per_step=2, start_compressing_after_num_steps=0)
        ddp = DDP(model, device_ids=[0], bucket_cap_mb=1000)  # one bucket
        state = PowerSGDState(cfg)
        ddp.register_comm_hook(state, powersgd_hook)
        psgd = None
        for step in range(4):
            gen = torch.Generator().manual_seed(100 * step + rank)
            x = torch.randn(32, 64, generator=gen).to(dev)
            ddp.zero_grad(set_to_none=True)
            ddp(x).square().mean().backward()
            ref.zero_grad(set_to_none=True)
            ref(x).square().mean().backward()
            if psgd is None:  # the replica batches the parameters in the hook codec's order
                (e,) = state._sets.values()
                by_id = {id(p): i for i, p in enumerate(model.parameters())}
                order = [by_id[pid] for pid in e["ids"]]
                ddp_params = [list(model.parameters())[i] for i in order]
                ref_params = [list(ref.parameters())[i] for i in order]
                psgd = PowerSGD(ref_params, cfg)
                resid = [torch.zeros_like(p) for p in ref_params]
            grads = [r + p.grad for r, p in zip(resid, ref_params)]
            outs = psgd.aggregate(grads)
            resid = grads
            got = [p.grad for p in ddp_params]
            for o, g in zip(outs, got):
                err = float((o - g).norm()) / max(float(o.norm()), 1e-30)
                assert err <= 1e-5, (rank, step, tuple(o.shape), err)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_ddp_hook_matches_reference_flow():
    with tempfile.TemporaryDirectory() as td:
        torch.multiprocessing.spawn(_worker, args=(2, os.path.join(td, "init")), nprocs=2, join=True)
