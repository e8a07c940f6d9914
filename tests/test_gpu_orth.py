"""GPU parity of the rank > 1 orthonormalisation (reference orthogonalization.py:8,
torch.linalg.qr = LAPACK geqrf + orgqr) INCLUDING the state it leaves behind.

Outputs and residuals are invariant to the column signs of the orthonormal factor, so the
other parity tests cannot see them; the P/Q state buffers can. The Cholesky-QR kernel
(k_orth_chol) reconstructs LAPACK's signs; the Householder fallback (rank-deficient and
zero panels) is LAPACK's own recursion. Both are checked against the CPU oracle's state
after one step (tolerance 1e-5 absolute on orthonormal columns)."""
import os

import pytest
import torch

from oracle import powersgd_oracle as O
from parity_log import check
from powersgd_amd import Config, PowerSGD
from powersgd_amd.workloads import hash_tensors

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")

SHAPES = [(64, 64), (300, 8, 3, 3), (8, 8), (1024, 256), (96, 4608), (5, 700), (2048, 512)]


@pytest.mark.parametrize("rank", [2, 3, 4, 5, 8, 12, 16, 24, 32])
@pytest.mark.parametrize("chol", ["1", "0"])
def test_state_signs_match_lapack(rank, chol):
    old = os.environ.get("PSGD_ORTH_CHOL")
    os.environ["PSGD_ORTH_CHOL"] = chol
    try:
        psgd = PowerSGD([torch.zeros(s, device=DEV) for s in SHAPES], Config(rank, 0.1, 1, 0))
        ora = O.policy_init([torch.zeros(s) for s in SHAPES], rank, 0.1, 1, 0)
        ora.codec.p_flat.copy_(psgd._powersgd._ps_buffer.cpu())
        ora.codec.q_flat.copy_(psgd._powersgd._qs_buffer.cpu())
        g = [torch.from_numpy(f) for f in hash_tensors(SHAPES, seed=17)]
        gd = [x.to(DEV) for x in g]
        psgd.aggregate(gd)  # step 0, one even iteration: P <- Q factor of qr(P)
        O.policy_step(ora, [x.clone() for x in g])
        torch.cuda.synchronize()
        p_gpu = psgd._powersgd._ps_buffer.cpu()
        check(float((p_gpu - ora.codec.p_flat).abs().max()), 1e-5, "orth_state", rank, chol)
    finally:
        if old is None:
            os.environ.pop("PSGD_ORTH_CHOL", None)
        else:
            os.environ["PSGD_ORTH_CHOL"] = old


def _structure_(view, kind, rank):
    """Give every P panel [B, n, r] a column LAPACK leaves unreflected (zero trailing
    sub-column: xnorm == 0, tau = 0, beta = alpha, so no sign flip)."""
    r = view.shape[2]
    if kind == "trapezoid":  # upper trapezoidal, mixed-sign diagonal: every column
        view[:, r:, :] = 0.0
        view.copy_(torch.triu(view))
        sign = torch.tensor([(-1.0) ** (j + rank) for j in range(r)])
        view.copy_(view.abs() * torch.where(torch.eye(view.shape[1], r) > 0, sign, torch.ones(r)))
    else:  # only column 0 = -2 e_0; the others stay random
        view[:, :, 0] = 0.0
        view[:, 0, 0] = -2.0


@pytest.mark.parametrize("rank", [2, 3, 4, 8, 16, 32])
@pytest.mark.parametrize("kind", ["trapezoid", "col0"])
@pytest.mark.parametrize("chol", ["1", "0"])
def test_unreflected_columns_match_lapack(rank, kind, chol):
    """the Cholesky-QR sign reconstruction assumed beta = -sign(alpha) for
    every column but the last; a zero trailing sub-column (tau = 0) must keep LAPACK's
    sign. Such panels are routed to the Householder recursion (k_orth_chol ok = false)."""
    old = os.environ.get("PSGD_ORTH_CHOL")
    os.environ["PSGD_ORTH_CHOL"] = chol
    try:
        psgd = PowerSGD([torch.zeros(s, device=DEV) for s in SHAPES], Config(rank, 0.1, 1, 0))
        ora = O.policy_init([torch.zeros(s) for s in SHAPES], rank, 0.1, 1, 0)
        for v in ora.codec.p_views:
            _structure_(v, kind, rank)
        psgd._powersgd._ps_buffer.copy_(ora.codec.p_flat.to(DEV))
        ora.codec.q_flat.copy_(psgd._powersgd._qs_buffer.cpu())
        g = [torch.from_numpy(f) for f in hash_tensors(SHAPES, seed=29)]
        psgd.aggregate([x.to(DEV) for x in g])
        O.policy_step(ora, [x.clone() for x in g])
        torch.cuda.synchronize()
        p_gpu = psgd._powersgd._ps_buffer.cpu()
        err = float((p_gpu - ora.codec.p_flat).abs().max())
        check(err, 1e-5, "orth_unreflected", kind, rank, chol)
    finally:
        if old is None:
            os.environ.pop("PSGD_ORTH_CHOL", None)
        else:
            os.environ["PSGD_ORTH_CHOL"] = old


@pytest.mark.parametrize("rank", [2, 4, 16, 32])
def test_zero_and_rank_deficient_panels(rank):
    """Zero gradients make the next factor zero (Householder fallback: identity columns);
    a rank-1 gradient makes it rank deficient."""
    shapes = [(64, 32), (64, 32), (128, 96)]
    psgd = PowerSGD([torch.zeros(s, device=DEV) for s in shapes], Config(rank, 0.1, 2, 0))
    ora = O.policy_init([torch.zeros(s) for s in shapes], rank, 0.1, 2, 0)
    ora.codec.p_flat.copy_(psgd._powersgd._ps_buffer.cpu())
    ora.codec.q_flat.copy_(psgd._powersgd._qs_buffer.cpu())
    u = torch.from_numpy(hash_tensors([(128, 1)], seed=3)[0])
    v = torch.from_numpy(hash_tensors([(1, 96)], seed=4)[0])
    g = [torch.zeros(64, 32), torch.zeros(64, 32), u @ v]
    for t in range(2):
        gd = [x.to(DEV) for x in g]
        gc = [x.clone() for x in g]
        outs = psgd.aggregate(gd)
        oc = O.policy_step(ora, gc)
        torch.cuda.synchronize()
        for i, x in enumerate(g):
            scale = max(float(x.norm()), 1.0)
            assert float((outs[i].cpu() - oc[i]).norm()) / scale <= 1e-5, (t, i)
            assert float((gd[i].cpu() - gc[i]).norm()) / scale <= 1e-5, (t, i)
        g = [r.cpu() + x for r, x in zip(gd, g)]


@pytest.mark.parametrize("rank", [2, 4])
@pytest.mark.parametrize("k", [2048, 2049, 4096, 4097, 5120, 5121, 11264, 11265])
def test_panel_length_instances(rank, k):
    """k_orth_chol picks its load-batch instance from the launch's longest panel (rank 4: 4-row
    batches up to 2048 rows, 10-row register-resident batches for 4097-5120; rank 2: 22-row
    batches for 4097-11264; the default batch otherwise). Panels at each side of every boundary,
    beside short panels of the same launch, against the oracle's LAPACK state: step 0
    orthonormalises the P panels (k rows), step 1 (I = 1, alternating) the Q panels."""
    shapes = [(k, 16), (16, k), (64, 8), (5, 40)]
    psgd = PowerSGD([torch.zeros(s, device=DEV) for s in shapes], Config(rank, 0.1, 1, 0))
    ora = O.policy_init([torch.zeros(s) for s in shapes], rank, 0.1, 1, 0)
    ora.codec.p_flat.copy_(psgd._powersgd._ps_buffer.cpu())
    ora.codec.q_flat.copy_(psgd._powersgd._qs_buffer.cpu())
    for t in range(2):
        g = [torch.from_numpy(f) for f in hash_tensors(shapes, seed=41 + t)]
        psgd.aggregate([x.to(DEV) for x in g])
        O.policy_step(ora, [x.clone() for x in g])
        torch.cuda.synchronize()
        # 1e-5 of the buffer's largest entry: the orthonormalised factor (entries <= 1) and the
        # other one, the raw product of that step (entries up to ~sqrt(k))
        for name, gpu, ref in (("p", psgd._powersgd._ps_buffer, ora.codec.p_flat),
                               ("q", psgd._powersgd._qs_buffer, ora.codec.q_flat)):
            err = float((gpu.cpu() - ref).abs().max()) / max(1.0, float(ref.abs().max()))
            check(err, 1e-5, "orth_panel_len_" + name, rank, k, t)
