"""Single-product kernel checks: ONE compress call (one power-iteration product) on one
matrix, against torch fp64. Each shape exercises one tile path of the products:
full-width row layout (m >= 129, m % 4 == 0), narrow lane-sum strips (m <= 128), scalar
columns (m % 4 != 0), small/ragged row counts, several strips and chunks.

Reference semantics (powersgd.py:186-197): in-factor X = orthonormalise(state), out =
G^T X (even parity) or G X (odd parity); the out-factor state buffer receives it."""
import pytest
import torch

from oracle import powersgd_oracle as O
from powersgd_amd import _lib

pytestmark = pytest.mark.gpu

SHAPES = [(3, 200), (64, 16), (37, 53), (120, 40), (8, 16), (32, 8), (256, 64), (256, 1152),
          (300, 1000), (1000, 300), (512, 4608), (4608, 512), (2, 2048), (2048, 3)]


def _run(shape, rank, even):
    dev = torch.device("cuda:0")
    n, m = shape
    r = min(rank, n, m)
    plan = _lib.Plan([shape], rank, 1, 0)
    pn, qn = plan.factor_numel()
    gen = torch.Generator().manual_seed(n * 7919 + m)
    g = torch.randn(shape, generator=gen, dtype=torch.float64)
    p0 = torch.randn(pn, generator=gen, dtype=torch.float64)
    q0 = torch.randn(qn, generator=gen, dtype=torch.float64)
    P = p0.float().to(dev)
    Q = q0.float().to(dev)
    ws = torch.empty(plan.workspace_bytes(), dtype=torch.uint8, device=dev)
    plan.bind(0, P.data_ptr(), Q.data_ptr(), ws.data_ptr())
    gd = g.float().to(dev)
    step = 0 if even else 1  # parity (step * iters + it) % 2 with iters = 1, it = 0
    plan.compress(_lib.ptr_array([gd.data_ptr()]), step, 0, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    xin = (p0 if even else q0).float().view(1, n if even else m, r)
    O.orthonormalise_(xin)  # the oracle's LAPACK-convention orthonormalisation
    x = xin[0].double()
    want = g.t() @ x if even else g @ x
    got = (Q if even else P).cpu().double().view(m if even else n, r)
    scale = float(g.norm() * x.norm()) + 1e-30
    return float((got - want).norm()) / scale


@pytest.mark.parametrize("rank", [1, 2, 4, 8])
@pytest.mark.parametrize("shape", SHAPES)
def test_single_product_odd(shape, rank):
    err = _run(shape, rank, even=False)
    assert err <= 1e-6, (shape, rank, err)


@pytest.mark.parametrize("rank", [1, 2, 4, 8])
@pytest.mark.parametrize("shape", SHAPES)
def test_single_product_even(shape, rank):
    err = _run(shape, rank, even=True)
    assert err <= 1e-6, (shape, rank, err)
