"""GPU parity of the folded Q orthonormalisation of the projection form (k_reduce's per-item
Gram partials + k_orth_chain, powersgd_amd/csrc/psgd_small.hip).

Two-iteration rank-2/4 plans at world size 1 orthonormalise the even iteration's Q from Gram
partials the reduction left, one workgroup per (panel, 1024-row slice). Pinned against:
* the oracle (bit-identical to the reference), per step from the same P/Q state, outputs,
  residuals AND the reference-visible P/Q state, at the per-step tolerance of
  tests/test_gpu_parity.py (1e-5 of the input norm);
* the unfolded plan (PSGD_QFOLD=0 at plan creation: k_orth_chol reads the panel itself),
  same tolerance, free-running over several steps;
* a zero matrix (its Q panel is zero: the chain rejects it and slice 0 runs the Householder
  recursion, LAPACK's identity columns) beside panels long enough for several slices.
"""
import os

import pytest
import torch

from oracle import powersgd_oracle as O
from powersgd_amd import Config, PowerSGD
from powersgd_amd.workloads import hash_tensors
from parity_log import check

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL = 1e-5

# Q panels of 32 .. 4608 rows (1 .. 5 slices of 1024 rows); n >= 2 r everywhere
SHAPES = [(64, 32), (96, 4608), (128, 1152), (64, 64), (257, 2048), (512, 128, 3, 3)]


def _make(shapes, rank, qfold):
    old = os.environ.get("PSGD_QFOLD")
    os.environ["PSGD_QFOLD"] = "1" if qfold else "0"
    try:
        return PowerSGD([torch.zeros(s, device=DEV) for s in shapes], Config(rank, 0.5, 2, 0))
    finally:
        if old is None:
            del os.environ["PSGD_QFOLD"]
        else:
            os.environ["PSGD_QFOLD"] = old


def _rel(a, b, scale):
    return float((a.double().cpu() - b.double().cpu()).norm()) / max(float(scale.double().norm()), 1e-30)


@pytest.mark.parametrize("rank", [2, 4])
def test_folded_q_orth_vs_oracle_per_step(rank):
    grads0 = [torch.from_numpy(x) for x in hash_tensors(SHAPES, seed=11 + rank)]
    grads0[0].zero_()  # zero panel: the Householder fallback in slice 0
    psgd = _make(SHAPES, rank, True)
    ora = O.policy_init([torch.zeros(s) for s in SHAPES], rank, 0.5, 2, 0)
    for step in range(3):
        # the reference's own state before every step (per-step parity)
        ora.codec.p_flat.copy_(psgd._powersgd._ps_buffer.cpu())
        ora.codec.q_flat.copy_(psgd._powersgd._qs_buffer.cpu())
        gd = [g.to(DEV) for g in grads0]
        gc = [g.clone() for g in grads0]
        outs = psgd.aggregate(gd)
        oc = O.policy_step(ora, gc)
        torch.cuda.synchronize()
        for i, g in enumerate(grads0):
            scale = g if float(g.norm()) > 0 else torch.ones(1)
            check(max(_rel(outs[i], oc[i], scale), _rel(gd[i], gc[i], scale)), TOL, rank, step, i)
        # the reference-visible state (orthonormal Q, P = G X - P_0 R'^T): absolute, the
        # factors are O(1) per column
        ep = float((psgd._powersgd._ps_buffer.cpu() - ora.codec.p_flat).abs().max())
        eq = float((psgd._powersgd._qs_buffer.cpu() - ora.codec.q_flat).abs().max())
        pmax = float(ora.codec.p_flat.abs().max())
        check(eq, 1e-5, rank, step, "q_state")
        check(ep / max(pmax, 1.0), 1e-5, rank, step, "p_state")


@pytest.mark.parametrize("rank", [2, 4])
def test_folded_q_orth_vs_unfolded_free_running(rank):
    grads0 = [torch.from_numpy(x) for x in hash_tensors(SHAPES, seed=23 + rank)]
    a = _make(SHAPES, rank, True)
    b = _make(SHAPES, rank, False)
    b._powersgd._ps_buffer.copy_(a._powersgd._ps_buffer)
    b._powersgd._qs_buffer.copy_(a._powersgd._qs_buffer)
    res_a = [g.to(DEV) for g in grads0]
    res_b = [g.to(DEV) for g in grads0]
    for step in range(4):
        ga = [r + g.to(DEV) for r, g in zip(res_a, grads0)]
        gb = [r + g.to(DEV) for r, g in zip(res_b, grads0)]
        inputs = [x.clone() for x in ga]
        oa = a.aggregate(ga)
        ob = b.aggregate(gb)
        torch.cuda.synchronize()
        for i in range(len(SHAPES)):
            # free-running: warm-start amplification (tolerance of the parity suite)
            check(max(_rel(oa[i], ob[i], inputs[i]), _rel(ga[i], gb[i], inputs[i])), 1e-4, rank, step, i)
        res_a, res_b = ga, gb
