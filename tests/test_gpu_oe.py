"""The odd-even pass (k_final_oe, psgd_plan.cpp oe_at): at rank 1, world size 1 and num_iters_per_step
>= 3, an odd power iteration followed by an even one (reference powersgd.py:172-202 twice: P_k =
G_k X_k, G_{k+1} = G_k - P_k X_k^T, Q_{k+1} = G_{k+1}^T orth(P_k)) runs as ONE gradient pass: the
row pass that forms P_k also accumulates the next product's column partials on the raw P_k, and
the reduction divides by the joint norm of P_k (orthogonalization.py:5-6) from the pass's sums
of squares. Checked per step against the CPU oracle (bit-identical to the reference) from the
same state, free-running over several steps, for even- and odd-start steps (I = 3 alternates),
multi-matrix shape groups (the joint norm couples them) and ragged shapes; and against the same
plan with the pass disabled (PSGD_OE=0)."""
import os

import pytest
import torch

from oracle import powersgd_oracle as O
from parity_log import check
from powersgd_amd import Config, PowerSGD
from powersgd_amd.workloads import hash_tensors

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")

SHAPES = [(64, 96), (64, 96), (64, 96), (128, 64), (200, 48), (96,), (300, 20, 3, 3), (4096, 512)]


def _rel(a, b, g):
    return float((a.double().cpu() - b.double().cpu()).norm()) / max(float(g.double().norm()), 1e-30)


def _make(iters, oe=True):
    old = os.environ.get("PSGD_OE")
    os.environ["PSGD_OE"] = "1" if oe else "0"
    try:
        return PSGD([torch.zeros(s, device=DEV) for s in SHAPES], Config(1, 2, iters, 0))
    finally:
        if old is None:
            del os.environ["PSGD_OE"]
        else:
            os.environ["PSGD_OE"] = old


PSGD = PowerSGD


@pytest.mark.parametrize("iters", [3, 4, 5])
def test_odd_even_pass_vs_oracle(iters):
    psgd = _make(iters)
    plan = psgd._powersgd._plan
    # the pass is taken on every odd iteration that has an even one after it
    for step in range(2):
        for it in range(iters):
            want = it >= 1 and it + 1 < iters and (step * iters + it) % 2 == 1
            assert plan.odd_even(step, it) == want, (step, it)
    ora = O.policy_init([torch.zeros(s) for s in SHAPES], 1, 2, iters, 0)
    ora.codec.p_flat.copy_(psgd._powersgd._ps_buffer.cpu())
    ora.codec.q_flat.copy_(psgd._powersgd._qs_buffer.cpu())
    res_d = [torch.zeros(s, device=DEV) for s in SHAPES]
    res_c = [torch.zeros(s) for s in SHAPES]
    for t in range(4):
        new = [torch.from_numpy(f) for f in hash_tensors(SHAPES, seed=4100 + t)]
        gd = [r + x.to(DEV) for r, x in zip(res_d, new)]
        gc = [r + x for r, x in zip(res_c, new)]
        scale = [g.clone() for g in gc]
        od = psgd.aggregate(gd)
        oc = O.policy_step(ora, gc)
        torch.cuda.synchronize()
        for i, g in enumerate(scale):
            tol = 1e-6 if t == 0 else 1e-4
            check(_rel(od[i], oc[i], g), tol, iters, t, i, "out")
            check(_rel(gd[i], gc[i], g), tol, iters, t, i, "res")
        # the reference-visible state after the step: P / Q as the reference leaves them
        check(_rel(psgd._powersgd._ps_buffer, ora.codec.p_flat, ora.codec.p_flat), 1e-4 if t else 1e-5, iters, t, "P")
        check(_rel(psgd._powersgd._qs_buffer, ora.codec.q_flat, ora.codec.q_flat), 1e-4 if t else 1e-5, iters, t, "Q")
        res_d, res_c = gd, gc


def test_odd_even_pass_against_separate_passes():
    """Same plan with the pass disabled: the same outputs up to rounding, every step."""
    a, b = _make(4, True), _make(4, False)
    assert a._powersgd._plan.odd_even(0, 1) and not b._powersgd._plan.odd_even(0, 1)
    b._powersgd._ps_buffer.copy_(a._powersgd._ps_buffer)
    b._powersgd._qs_buffer.copy_(a._powersgd._qs_buffer)
    ra = [torch.zeros(s, device=DEV) for s in SHAPES]
    rb = [torch.zeros(s, device=DEV) for s in SHAPES]
    for t in range(3):
        new = [torch.from_numpy(f).to(DEV) for f in hash_tensors(SHAPES, seed=5100 + t)]
        ga = [r + x for r, x in zip(ra, new)]
        gb = [r + x for r, x in zip(rb, new)]
        scale = [g.clone() for g in ga]
        oa, ob = a.aggregate(ga), b.aggregate(gb)
        torch.cuda.synchronize()
        for i, g in enumerate(scale):
            check(_rel(oa[i], ob[i], g), 1e-6 if t == 0 else 1e-4, t, i, "out")
            check(_rel(ga[i], gb[i], g), 1e-6 if t == 0 else 1e-4, t, i, "res")
        ra, rb = ga, gb
