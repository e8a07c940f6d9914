"""fp64 gradients on the GPU (psgd_f64.hip) — the reference's own test dtype.

The reference runs its error-feedback test in float64 (tests/powersgd_test.py:37-55): it sets
torch's default dtype to float64, so its P/Q factors (powersgd.py:241-251) and every product are
fp64. Checked here:
* the reference-produced fixture F1_refmodel_r2_i3_mcr10_f64 (per step from the reference's own
  state, and free-running);
* a mirror of test_error_feedback_mechanism (out + residual == input) in fp64;
* the oracle (bit-identical to the reference) in fp64 on larger shapes, every rank bucket,
  several iterations, at world size 1 and over gloo at world size 2 (two processes on cuda:0);
* a float32 default dtype with fp64 gradients raises, as the reference's bmm does.
Tolerance: TOL_F64 = 1e-12 of the input norm per tensor (GPU Householder/partial-sum order vs
LAPACK/BLAS; measured errors are ~2e-16 on the reference fixture, logged by parity_log).
"""
import os
import tempfile

import numpy as np
import pytest
import torch

from golden_io import load, manifest, scenario_inputs
from oracle import powersgd_oracle as O
from parity_log import check
from powersgd_amd import Config, PowerSGD
from powersgd_amd.workloads import hash_tensors

pytestmark = pytest.mark.gpu
TOL_F64 = 1e-12
DEV = torch.device("cuda:0")
MAN = manifest()


def _rel(a, b, scale) -> float:
    return float((a.double().cpu() - torch.as_tensor(b).double()).norm()) / max(float(scale.double().norm()), 1e-300)


@pytest.fixture
def f64_default():
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    yield
    torch.set_default_dtype(prev)


def _inject(psgd, p, q, steps):
    psgd._powersgd._ps_buffer.copy_(torch.from_numpy(np.ascontiguousarray(p)).to(DEV))
    psgd._powersgd._qs_buffer.copy_(torch.from_numpy(np.ascontiguousarray(q)).to(DEV))
    psgd.step_counter, psgd._powersgd.step_counter = int(steps[0]), int(steps[1])


@pytest.mark.parametrize("mode", ["per_step", "free_running"])
def test_reference_fp64_golden(mode, f64_default):
    name = "refmodel_r2_i3_mcr10_f64"
    meta = MAN["scenarios"][name]
    want = load("F1_" + name)
    shapes = [tuple(s) for s in meta["shapes"]]
    psgd = PowerSGD([torch.zeros(s, device=DEV) for s in shapes],
                    Config(meta["rank"], meta["mcr"], meta["iters"], meta["start"]))
    assert psgd._powersgd._ps_buffer.dtype == torch.float64
    assert psgd.is_compressed_mask == list(want["mask"])
    _inject(psgd, want["p0"], want["q0"], (0, 0))
    res = [torch.zeros(s) for s in shapes]
    for t in range(meta["steps"]):
        if mode == "per_step" and t > 0:
            _inject(psgd, want[f"s{t-1}_p"], want[f"s{t-1}_q"], want[f"s{t-1}_step"])
            res = [torch.from_numpy(want[f"s{t-1}_res_{i}"]) for i in range(len(shapes))]
        inputs = scenario_inputs(meta, t, res, dtype=torch.float64)
        grads = [g.to(DEV) for g in inputs]
        outs = psgd.aggregate(grads)
        torch.cuda.synchronize()
        for i, g in enumerate(inputs):
            assert outs[i].dtype == torch.float64
            check(_rel(outs[i], want[f"s{t}_out_{i}"], g), TOL_F64, name, mode, t, i, "out")
            check(_rel(grads[i], want[f"s{t}_res_{i}"], g), TOL_F64, name, mode, t, i, "res")
        res = [x.cpu() for x in grads]


def test_error_feedback_mechanism_fp64(f64_default):
    """tests/powersgd_test.py:37-55 verbatim in spirit: float64 default dtype, rank 2, I = 3."""
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Conv2d(3, 100, 3), torch.nn.ReLU(), torch.nn.Conv2d(100, 50, 5),
                                torch.nn.Linear(50, 1)).to(DEV)
    params = list(model.parameters())
    psgd = PowerSGD(params, Config(rank=2, min_compression_rate=10, start_compressing_after_num_steps=0,
                                   num_iters_per_step=3))
    grads = [torch.randn_like(p) for p in params]
    orig = [g.clone() for g in grads]
    avg = psgd.aggregate(grads)
    for o, a, b in zip(orig, avg, grads):
        assert o.allclose(a + b)


SHAPES = [(300, 200), (64, 1000), (1000, 64), (128, 8, 3, 3), (40,), (64, 32), (64, 32), (1, 50)]


@pytest.mark.parametrize("rank,iters", [(1, 2), (2, 1), (4, 3), (8, 2), (16, 2), (32, 1), (1, 4)])
def test_fp64_vs_oracle(rank, iters, f64_default):
    params = [torch.zeros(s, device=DEV) for s in SHAPES]
    psgd = PowerSGD(params, Config(rank, 0.5, iters, 0))
    ora = O.policy_init([torch.zeros(s) for s in SHAPES], rank, 0.5, iters, 0)
    assert ora.codec.p_flat.dtype == torch.float64
    ora.codec.p_flat.copy_(psgd._powersgd._ps_buffer.cpu())
    ora.codec.q_flat.copy_(psgd._powersgd._qs_buffer.cpu())
    res_d = [torch.zeros(s, device=DEV) for s in SHAPES]
    res_c = [torch.zeros(s) for s in SHAPES]
    for t in range(3):
        new = [torch.from_numpy(f).double() for f in hash_tensors(SHAPES, seed=90 + t)]
        gd = [r + x.to(DEV) for r, x in zip(res_d, new)]
        gc = [r + x for r, x in zip(res_c, new)]
        scale = [g.clone() for g in gc]
        od = psgd.aggregate(gd)
        oc = O.policy_step(ora, gc)
        torch.cuda.synchronize()
        for i, g in enumerate(scale):
            check(_rel(od[i], oc[i], g), TOL_F64, rank, iters, t, i, "out")
            check(_rel(gd[i], gc[i], g), TOL_F64, rank, iters, t, i, "res")
        res_d, res_c = gd, gc


def test_fp64_with_fp32_default_dtype_raises():
    with pytest.raises(RuntimeError, match="expected scalar type Double"):
        PowerSGD([torch.zeros(64, 32, device=DEV, dtype=torch.float64)], Config(1, 0.5, 1, 0))


def _w2_worker(rank_id, world, initfile):
    torch.set_default_dtype(torch.float64)
    torch.distributed.init_process_group("gloo", init_method=f"file://{initfile}", rank=rank_id, world_size=world)
    try:
        shapes = SHAPES
        psgd = PowerSGD([torch.zeros(s, device=DEV) for s in shapes], Config(2, 0.5, 2, 1))
        ora = O.policy_init([torch.zeros(s) for s in shapes], 2, 0.5, 2, 1)
        ora.codec.p_flat.copy_(psgd._powersgd._ps_buffer.cpu())
        ora.codec.q_flat.copy_(psgd._powersgd._qs_buffer.cpu())
        res_d = [torch.zeros(s, device=DEV) for s in shapes]
        res_c = [torch.zeros(s) for s in shapes]
        for t in range(3):
            new = [torch.from_numpy(f).double() for f in hash_tensors(shapes, seed=300 + 10 * t + rank_id)]
            gd = [r + x.to(DEV) for r, x in zip(res_d, new)]
            gc = [r + x for r, x in zip(res_c, new)]
            scale = [g.clone() for g in gc]
            od = psgd.aggregate(gd)
            oc = O.policy_step(ora, gc, world, lambda b: torch.distributed.all_reduce(b))
            torch.cuda.synchronize()
            for i, g in enumerate(scale):
                check(_rel(od[i], oc[i], g), TOL_F64, "w2", rank_id, t, i, "out")
                check(_rel(gd[i], gc[i], g), TOL_F64, "w2", rank_id, t, i, "res")
            res_d, res_c = gd, gc
        torch.distributed.barrier()
    finally:
        torch.distributed.destroy_process_group()


def test_fp64_world_size_2_vs_oracle():
    with tempfile.TemporaryDirectory() as td:
        torch.multiprocessing.spawn(_w2_worker, args=(2, os.path.join(td, "init")), nprocs=2, join=True)
