"""The DDP comm hook (powersgd_amd/ddp.py) at Llama scale: more than 2^31 gradient elements
(bf16), one training iteration through DistributedDataParallel with powersgd_hook. The bucket
plumbing is the native run table (include/psgd.h psgd_runs_*: 64-bit offsets, no index maps),
so nothing caps the element count.

Size-independent property checked at full size: every gradient here is a rank-1
matrix (the loss is sum_i s_i * sum(p_i), so dL/dp_i = s_i everywhere), which a rank-1 PowerSGD
step with two power iterations reproduces exactly up to rounding when each matrix is its own
shape group (the reference's rank-1 joint norm, orthogonalization.py:5-6, then normalises per
matrix): out = X0 X0^T G + (G - X0 X0^T G) = G, residual 0. So the averaged gradient DDP hands
back equals s_i and the error-feedback residual left in the state is ~0 (within bf16 rounding of
s_i). The uncompressed bias goes through the flat path unchanged."""
import os
import tempfile
import time

import pytest
import torch

pytestmark = pytest.mark.gpu

# 16 matrices [16384, 8192 + 64 i] (16 shape groups) + [1000]: 2.27e9 elements > 2^31, 4.5 GB
# of bf16 per copy
SHAPES = [(16384, 8192 + 64 * i) for i in range(16)] + [(1000,)]
SCALES = [0.5 + 0.125 * i for i in range(len(SHAPES))]  # exact in bf16


class _Model(torch.nn.Module):
    def __init__(self, dev):
        super().__init__()
        self.ps = torch.nn.ParameterList(
            [torch.nn.Parameter(torch.zeros(s, device=dev, dtype=torch.bfloat16)) for s in SHAPES])

    def forward(self, z):
        return sum(p.sum() * s for p, s in zip(self.ps, SCALES)) + z.sum()


def _worker(rank, initfile, q):
    from torch.nn.parallel import DistributedDataParallel as DDP

    from powersgd_amd import Config
    from powersgd_amd.ddp import PowerSGDState, powersgd_hook

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    # one RCCL rank: DDP and the codec's multi-GPU code path (the library's own communicator)
    torch.distributed.init_process_group("nccl", init_method=f"file://{initfile}", rank=0, world_size=1,
                                         device_id=dev)
    try:
        model = _Model(dev)
        params = list(model.parameters())
        assert sum(p.numel() for p in params) > 2 ** 31
        ddp = DDP(model, device_ids=[0], gradient_as_bucket_view=True)
        state = PowerSGDState(Config(rank=1, min_compression_rate=2, num_iters_per_step=2,
                                     start_compressing_after_num_steps=0), params=params)
        assert state.powersgd.is_compressed_mask == [True] * 16 + [False]
        ddp.register_comm_hook(state, powersgd_hook)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ddp(torch.zeros(1, device=dev)).backward()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        worst_avg = worst_res = 0.0
        for p, s, v in zip(params, SCALES, state.views):
            g = p.grad.float()
            worst_avg = max(worst_avg, float((g - s).abs().max()) / s)
            worst_res = max(worst_res, float(v.float().abs().max()) / s)
        q.put((worst_avg, worst_res, dt, len(state._runs)))
    finally:
        torch.distributed.destroy_process_group()


def test_ddp_hook_beyond_2_31_elements_bf16():
    ctx = torch.multiprocessing.get_context("spawn")
    q = ctx.SimpleQueue()
    with tempfile.TemporaryDirectory() as td:
        torch.multiprocessing.spawn(_worker, args=(os.path.join(td, "init"), q), nprocs=1, join=True)
    worst_avg, worst_res, dt, nbuckets = q.get()
    print(f"one DDP iteration, {sum(a * b for a, b in SHAPES[:16]) + 1000} bf16 elements: {dt * 1e3:.1f} ms, "
          f"{nbuckets} buckets, max rel |avg - g| {worst_avg:.2e}, max rel |residual| {worst_res:.2e}")
    assert nbuckets >= 1
    # bf16 storage of the average and the residual: a few ulps of s (2^-8 relative per ulp)
    assert worst_avg <= 2e-2 and worst_res <= 2e-2, (worst_avg, worst_res)
