"""The matrix-core even product of ranks 9-32 (k_even's even_seg_mfma: v_mfma_f32_16x16x4_f32
over 4-row x 64-column gradient quads, psgd_even.cuh) against the CPU oracle.

At rank buckets 16 / 32 the first iteration's product Q = G^T X takes the matrix cores for every
matrix with m % 4 == 0 and a 16-byte aligned gradient (8-byte for bf16), and the scalar-column
VALU form otherwise; both leave the same partial layout, so one plan mixes them. Covered: full
64-column strips, a ragged last strip (m = 200), a narrow matrix inside one strip (m = 40, and
m = 20: a 32-column strip), ragged row counts (4-row groups past the segment end), effective
ranks below the bucket (r = 12 in bucket 16, r = 20 in 32, and matrices whose r = min(rank, n,
m) is smaller still), an m % 4 != 0 matrix (fallback), a misaligned gradient view (fallback),
bf16 gradients, and many segments per strip (ResNet-50 shapes). One step (I = 2) from the same
state against the oracle within the stated fp32 tolerance (1e-5 of the input norm; bf16 4e-3),
and a bitwise rerun (fixed-order sums)."""
import pytest
import torch

from parity_log import check
from oracle import powersgd_oracle as O
from powersgd_amd import Config, PowerSGD
from powersgd_amd.workloads import hash_tensors, resnet50_shapes

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL_STEP = 1e-5
TOL_BF16 = 4e-3

SHAPES = [(300, 200), (64, 1000), (1000, 64), (2048, 576), (96, 40), (50, 20), (333, 148), (200, 150),
          (40,), (130, 16, 3, 3)]


def _rel(a, b, scale) -> float:
    return float((a.double().cpu() - b.double().cpu()).norm()) / max(float(scale.double().norm()), 1e-30)


def _one_step(shapes, rank, dt=torch.float32, misalign=()):
    psgd = PowerSGD([torch.zeros(s, device=DEV, dtype=dt) for s in shapes], Config(rank, 0.1, 2, 0))
    p0 = psgd._powersgd._ps_buffer.clone()
    q0 = psgd._powersgd._qs_buffer.clone()
    new = [torch.from_numpy(f) for f in hash_tensors(shapes, seed=131 + rank)]
    gin = [g.to(DEV).to(dt) for g in new]
    ora = O.policy_init([torch.zeros(s) for s in shapes], rank, 0.1, 2, 0)
    ora.codec.p_flat.copy_(p0.cpu())
    ora.codec.q_flat.copy_(q0.cpu())
    gc = [g.float().cpu() for g in gin]
    scale = [g.clone() for g in gc]
    oc = O.policy_step(ora, gc)
    runs = []
    for _ in range(2):
        psgd._powersgd._ps_buffer.copy_(p0)
        psgd._powersgd._qs_buffer.copy_(q0)
        psgd.step_counter = psgd._powersgd.step_counter = 0
        gd = []
        for i, g in enumerate(gin):
            if i in misalign:  # a view one element into a larger buffer: not 16-byte aligned
                buf = torch.empty(g.numel() + 1, device=DEV, dtype=dt)
                v = buf[1:].view(g.shape)
                v.copy_(g)
                assert v.data_ptr() % 16 != 0
                gd.append(v)
            else:
                gd.append(g.clone())
        od = psgd.aggregate(gd)
        torch.cuda.synchronize()
        runs.append([o.clone() for o in od] + [g.clone() for g in gd] +
                    [psgd._powersgd._ps_buffer.clone(), psgd._powersgd._qs_buffer.clone()])
        tol = TOL_BF16 if dt == torch.bfloat16 else TOL_STEP
        for i, g in enumerate(scale):
            check(_rel(od[i].float(), oc[i], g), tol, rank, str(dt), i, "out")
            check(_rel(gd[i].float(), gc[i], g), tol, rank, str(dt), i, "res")
    for x, y in zip(runs[0], runs[1]):
        assert torch.equal(x, y)


@pytest.mark.parametrize("rank", [12, 16, 20, 32])
def test_even_mfma_shapes(rank):
    _one_step(SHAPES, rank)


@pytest.mark.parametrize("rank", [16, 32])
def test_even_mfma_misaligned_fallback(rank):
    _one_step(SHAPES, rank, misalign=(0, 3))


@pytest.mark.parametrize("rank", [16, 32])
def test_even_mfma_bf16(rank):
    _one_step(SHAPES[:7], rank, dt=torch.bfloat16)


@pytest.mark.parametrize("rank", [16, 32])
def test_even_mfma_resnet50(rank):
    _one_step(resnet50_shapes(), rank)
