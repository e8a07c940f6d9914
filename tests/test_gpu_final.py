"""GPU parity of the fused final odd pass (k_final_odd, powersgd_amd/csrc/psgd_final.cuh).

When the last power iteration of a step is odd (P = G_k X), the library runs that
iteration and the final residual/output pass as ONE kernel that keeps gradient rows in
registers. These tests pin it three ways:
* against the CPU oracle (bit-identical to the reference) from the same P/Q state, per
  step, at the per-step tolerance of tests/test_gpu_parity.py (1e-5 of the input norm);
* against the unfused kernels (PSGD_FUSE_FINAL=0 at plan creation), same tolerance: only
  the summation order of P = G_k X differs;
* the world-size > 1 code path (psgd_compress writes the residual, psgd_decompress writes
  only the output with k_lowrank_out) driven at world size 1 through the C ABI, against
  the single-call psgd_aggregate.
Two-iteration rank-1/2/4 plans take the projection form in psgd_aggregate (output G X X^T,
residual G - G X X^T, P state G X - P_0 R'^T; exact algebra for I = 2 at world size 1, see
psgd_final.cuh): checked against the oracle at the same 1e-5, and against the K-term form
(PSGD_FIN_PROJ=0) through the unfused comparison.
Shapes cover every row-group form: sub-wave groups (m <= 256), one to four waves, several
register segments, bf16 rows, rank caps, and a matrix whose rows do not fill a batch.
"""
import os

import pytest
import torch

from oracle import powersgd_oracle as O
from powersgd_amd import Config, PowerSGD
from powersgd_amd.workloads import hash_tensors

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL = 1e-5

SHAPES = [(64, 64), (64, 64), (33, 20), (256, 64, 1, 1), (100, 3, 3, 3), (512, 128, 3, 3),
          (128, 1152), (96, 4608), (257, 2048), (9, 1000)]
# (n >= 2 r for every matrix: with n < 2 r the second iteration's panel P = G_1 X is rank
# deficient (G_1 = G_0 minus its rank-r projection has rank n - r < r), its Householder Q
# has columns fixed only by rounding noise, and the reference's own outputs are then not
# reproducible across BLAS implementations.)


def _rel(a, b, scale):
    return float((a.double().cpu() - b.double().cpu()).norm()) / max(float(scale.double().norm()), 1e-30)


def _make(shapes, rank, iters, dtype=torch.float32, fuse=True, proj=True):
    env = {"PSGD_FUSE_FINAL": "1" if fuse else "0", "PSGD_FIN_PROJ": "1" if proj else "0"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        psgd = PowerSGD([torch.zeros(s, device=DEV, dtype=dtype) for s in shapes],
                        Config(rank, 0.5, iters, 0))
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    return psgd


# rows of at most 2048 columns: every rank <= 2 instance fits (with three or more
# iterations the uncached-term kernel spills at wider rows, and the plan keeps those unfused)
NARROW = [s for s in SHAPES if int(torch.tensor(s[1:]).prod()) <= 2048]


# mode: "p" the default fused forms (projection form where it applies); "k": the projection form
# off (the K-term form at I = 2, ranks 1-2; rank 4 has no K-term form and stays unfused)
@pytest.mark.parametrize("rank,iters,narrow,mode", [
    (1, 2, False, "p"), (2, 2, False, "p"), (1, 1, False, "p"), (2, 1, False, "p"), (1, 3, False, "p"),
    (1, 4, False, "p"), (4, 2, False, "p"), (2, 3, False, "p"), (1, 3, True, "p"), (2, 4, True, "p"),
    (2, 2, True, "p"), (4, 2, False, "k"), (2, 2, False, "k"), (4, 2, True, "p"), (4, 1, False, "p"),
    (4, 1, True, "p")])
def test_fused_final_vs_oracle_and_unfused(rank, iters, narrow, mode):
    shapes = NARROW if narrow else SHAPES
    proj = mode != "k"
    fused = _make(shapes, rank, iters, fuse=True, proj=proj)
    plain = _make(shapes, rank, iters, fuse=False)
    plain._powersgd._ps_buffer.copy_(fused._powersgd._ps_buffer)
    plain._powersgd._qs_buffer.copy_(fused._powersgd._qs_buffer)
    n_fused = 0
    res = [torch.zeros(s) for s in shapes]
    for t in range(3):
        form = fused._powersgd._plan.fused_final(t)
        n_fused += bool(form)
        if form:  # 2 = projection form: exactly the two-iteration rank-2/4 register-panel plans
            assert (form == 2) == (proj and iters == 2 and rank in (1, 2, 4)), (form, t)
        ora = O.policy_init([torch.zeros(s) for s in shapes], rank, 0.5, iters, 0)
        ora.codec.p_flat.copy_(fused._powersgd._ps_buffer.cpu())
        ora.codec.q_flat.copy_(fused._powersgd._qs_buffer.cpu())
        ora.step = fused.step_counter
        ora.codec.step = fused._powersgd.step_counter
        fresh = [torch.from_numpy(f) for f in hash_tensors(shapes, seed=300 + t)]
        inputs = [r + f for r, f in zip(res, fresh)]
        g_f = [x.to(DEV) for x in inputs]
        g_p = [x.to(DEV) for x in inputs]
        g_c = [x.clone() for x in inputs]
        o_f = fused.aggregate(g_f)
        o_p = plain.aggregate(g_p)
        o_c = O.policy_step(ora, g_c)
        torch.cuda.synchronize()
        for i, x in enumerate(inputs):
            for name, a, b in (("out/oracle", o_f[i], o_c[i]), ("res/oracle", g_f[i], g_c[i]),
                               ("out/unfused", o_f[i], o_p[i]), ("res/unfused", g_f[i], g_p[i])):
                e = _rel(a, b, x)
                assert e <= TOL, (rank, iters, t, i, shapes[i], name, e)
            assert _rel(o_f[i] + g_f[i], x, x) <= 1e-6  # error-feedback identity (W = 1)
        res = [g.cpu() for g in g_f]
        # keep the unfused run on exactly the fused run's state (warm-start drift aside)
        plain._powersgd._ps_buffer.copy_(fused._powersgd._ps_buffer)
        plain._powersgd._qs_buffer.copy_(fused._powersgd._qs_buffer)
    expect_odd_last = sum(((t * iters + iters - 1) % 2) == 1 for t in range(3))
    projection = proj and iters == 2 and rank in (1, 2, 4)
    # configurations that must fuse (rank 4 fuses only in the projection form)
    if (narrow and rank <= 2) or (rank == 1 and iters <= 2) or projection:
        assert n_fused == expect_odd_last, (n_fused, expect_odd_last)


def test_fused_final_bf16():
    shapes = [(64, 2048), (96, 2304), (40, 64)]
    psgd = _make(shapes, 2, 2, dtype=torch.bfloat16)
    assert psgd._powersgd._plan.fused_final(0)
    ora = O.policy_init([torch.zeros(s) for s in shapes], 2, 0.5, 2, 0)
    ora.codec.p_flat.copy_(psgd._powersgd._ps_buffer.cpu())
    ora.codec.q_flat.copy_(psgd._powersgd._qs_buffer.cpu())
    g = [torch.from_numpy(f).to(DEV).to(torch.bfloat16) for f in hash_tensors(shapes, seed=9)]
    x = [t.float().cpu() for t in g]
    g_c = [t.clone() for t in x]
    outs = psgd.aggregate(g)
    o_c = O.policy_step(ora, g_c)
    torch.cuda.synchronize()
    for i in range(len(shapes)):
        assert _rel(outs[i].float(), o_c[i], x[i]) <= 4e-3
        assert _rel(g[i].float(), g_c[i], x[i]) <= 4e-3


@pytest.mark.parametrize("rank,iters", [(1, 2), (2, 2), (1, 1), (16, 2)])
def test_split_calls_match_aggregate(rank, iters):
    """psgd_compress (fused last iteration writes the residual) + psgd_decompress
    (k_lowrank_out writes the output): the world-size > 1 sequence, at world size 1."""
    shapes = SHAPES
    # the split calls have no projection form: compare with psgd_aggregate's K-term form
    a = _make(shapes, rank, iters, proj=False)
    b = _make(shapes, rank, iters, proj=False)
    b._powersgd._ps_buffer.copy_(a._powersgd._ps_buffer)
    b._powersgd._qs_buffer.copy_(a._powersgd._qs_buffer)
    ca, cb = a._powersgd, b._powersgd
    stream = torch.cuda.current_stream().cuda_stream
    for t in range(2):
        grads = [torch.from_numpy(f).to(DEV) for f in hash_tensors(shapes, seed=40 + t)]
        ga = [g.clone() for g in grads]
        gb = [g.clone() for g in grads]
        oa = a.aggregate(ga)
        comp = [g for g, m in zip(gb, b.is_compressed_mask) if m]
        cb._table.fill(comp)
        ptrs = cb._table.comp_addr()
        out = torch.empty(cb._out_numel, device=DEV)
        for it in range(iters):
            cb._plan.compress(ptrs, t, it, stream)
        cb._plan.decompress(ptrs, out.data_ptr(), t, 1, stream)
        cb.step_counter += 1
        b._allreduce.aggregate([g for g, m in zip(gb, b.is_compressed_mask) if not m])
        torch.cuda.synchronize()
        offs = cb._plan.output_offsets()
        k = 0
        for i, (g, m) in enumerate(zip(grads, a.is_compressed_mask)):
            if not m:
                continue
            ob = out[offs[k]:offs[k] + g.numel()].view(g.shape)
            k += 1
            assert _rel(oa[i], ob, g) <= 1e-6, (t, i, "out")
            assert _rel(ga[i], gb[i], g) <= 1e-6, (t, i, "res")


@pytest.mark.parametrize("cfg,form", [("cfg1_1024sq_r1", 2), ("cfg2_resnet50_r1", 2), ("cfg3_resnet50_r4", 2),
                                      ("cfg5_lstm_r1_i4", 1)])
def test_baseline_configs_take_the_fused_forms(cfg, form):
    """The BASELINE configurations run the fused final pass at world size 1 (K-term form, or the
    projection form at rank 4): an instance that stops fitting two waves per SIMD without scratch
    (e.g. after a kernel change) silently falls back to the unfused kernels — caught here."""
    from powersgd_amd.workloads import CONFIGS

    c = CONFIGS[cfg]
    psgd = PowerSGD([torch.zeros(s, device=DEV) for s in c["shapes"]], Config(c["rank"], c["mcr"], c["iters"], 0))
    assert [psgd._powersgd._plan.fused_final(t) for t in range(2)] == [form, form], cfg
