"""Host-memory PowerSGD (powersgd_amd/host.py): CPU gradients in, CPU outputs out, the codec
on the GPU, bins of whole shape groups pipelined over streams. Checked against the CPU
oracle (bit-identical to the reference, including the reference's CPU-generator P/Q
initialisation) over several error-feedback steps; two shards on cuda:0 stand in for two
GPUs (the sharding and the state scatter are the same code). Tolerance: the free-running
bound of tests/test_gpu_parity.py (1e-4 of the input norm over <= 4 steps)."""
import pytest
import torch

from oracle import powersgd_oracle as O
from powersgd_amd import Config
from powersgd_amd.host import HostPowerSGD
from powersgd_amd.workloads import hash_tensors

pytestmark = pytest.mark.gpu
TOL = 1e-4

SHAPES = [(64, 32, 3, 3), (64, 32, 3, 3), (64, 32, 3, 3), (128, 64), (64,), (256, 64, 1, 1), (100, 3, 3, 3),
          (512, 256), (32,), (10, 512), (512, 256)]


@pytest.mark.parametrize("rank,iters,pin,devices,chunks",
                         [(1, 2, True, [0, 0], 2), (2, 1, False, [0], 3), (4, 2, True, [0], 1), (1, 3, False, [0, 0], 1)])
def test_host_pipeline_matches_reference(rank, iters, pin, devices, chunks):
    params = [torch.zeros(s) for s in SHAPES]
    cfg = Config(rank, 2, iters, 1)  # one warm-up step (plain average) first
    host = HostPowerSGD(params, cfg, devices=devices, chunks=chunks)
    ora = O.policy_init([torch.zeros(s) for s in SHAPES], rank, 2, iters, 1)
    if pin:
        host.pin_gradients(params)
    res_h = [torch.zeros(s) for s in SHAPES]
    res_o = [torch.zeros(s) for s in SHAPES]
    for t in range(4):
        fresh = [torch.from_numpy(f) for f in hash_tensors(SHAPES, seed=900 + t)]
        if pin:  # autograd-style accumulation into the pinned p.grad views
            for p, f in zip(params, fresh):
                p.grad.add_(f)
            g_h = [p.grad for p in params]
        else:
            g_h = [r + f for r, f in zip(res_h, fresh)]
        g_o = [r + f for r, f in zip(res_o, fresh)]
        inputs = [x.clone() for x in g_o]
        out_h = host.aggregate(g_h)
        out_o = O.policy_step(ora, g_o)
        for i, x in enumerate(inputs):
            scale = max(float(x.norm()), 1e-30)
            eo = float((out_h[i] - out_o[i]).norm()) / scale
            er = float((g_h[i] - g_o[i]).norm()) / scale
            assert eo <= TOL and er <= TOL, (t, i, SHAPES[i], eo, er)
        res_h = [g.clone() for g in g_h]
        res_o = g_o
        del out_h


def test_held_outputs_are_not_overwritten():
    params = [torch.zeros(s) for s in SHAPES]
    host = HostPowerSGD(params, Config(1, 2, 2, 0), devices=[0])
    g = [torch.from_numpy(f) for f in hash_tensors(SHAPES, seed=1)]
    first = host.aggregate([x.clone() for x in g])
    keep = [o.clone() for o in first]
    host.aggregate([x.clone() * 3 for x in g])
    for a, b in zip(first, keep):
        assert torch.equal(a, b)


@pytest.mark.parametrize("pin,skip_zero", [(False, False), (True, False), (True, True)])
def test_device_residual_variant_equals_reference_contract(pin, skip_zero):
    """residual="device" (outputs-only D2H; the caller hands FRESH gradients each step and the
    residual stays on the GPU) returns bitwise the outputs of the reference contract (residual
    back in the caller's tensors, next gradient accumulated onto it), and the same residual."""
    cfg = Config(2, 2, 2, 1)
    p_ref = [torch.zeros(s) for s in SHAPES]
    p_dev = [torch.zeros(s) for s in SHAPES]
    ref = HostPowerSGD(p_ref, cfg, devices=[0, 0], chunks=2)
    dev = HostPowerSGD(p_dev, cfg, devices=[0, 0], chunks=2, residual="device")
    if pin:
        dev.pin_gradients(p_dev)
    res = [torch.zeros(s) for s in SHAPES]
    for t in range(4):
        fresh = [torch.from_numpy(f) for f in hash_tensors(SHAPES, seed=300 + t)]
        g_ref = [r + f for r, f in zip(res, fresh)]
        if pin:
            for p, f in zip(p_dev, fresh):
                if not skip_zero:  # skip_zero: a loop that forgets zero_grad()
                    p.grad.zero_()
                p.grad.add_(f)  # zero_grad + backward
            g_dev = [p.grad for p in p_dev]
        else:
            g_dev = [f.clone() for f in fresh]
        out_ref = ref.aggregate(g_ref)
        out_dev = dev.aggregate(g_dev)
        for i in range(len(SHAPES)):
            assert torch.equal(out_ref[i], out_dev[i]), (t, i)
            # every input is consumed: compressed ones now live in the device residual
            assert not bool(g_dev[i].any()), (t, i)
        r_dev = dev.residual()
        for i, c in enumerate(ref.is_compressed_mask):
            if c:
                assert torch.equal(r_dev[i], g_ref[i]), (t, i)
        res = [g if c else torch.zeros_like(g) for g, c in zip(g_ref, ref.is_compressed_mask)]
