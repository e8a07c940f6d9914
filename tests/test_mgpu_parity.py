"""CPU tests of bench.py's cross-GPU parity check (N > 1): the W-worker oracle
(oracle/multiworker.py) against the reference's own gloo goldens, and the whole
gather-and-compare pipeline over a 2-process gloo group (the product step replaced by the
reference restatement over gloo, so a correct pipeline reports zero error and a corrupted
rank is caught)."""
import os
import tempfile

import numpy as np
import pytest
import torch

import bench
from golden_io import load, manifest, scenario_inputs
from oracle import multiworker as MW
from oracle import powersgd_oracle as O

MAN = manifest()


@pytest.mark.parametrize("key", sorted(MAN["multi"]))
def test_threaded_workers_match_reference_gloo_goldens(key):
    info = MAN["multi"][key]
    meta = MAN["scenarios"][info["scenario"]]
    world = info["world"]
    want = load("F2_" + key)
    shapes = [tuple(s) for s in meta["shapes"]]
    states = []
    for w in range(world):
        st = O.policy_init([torch.zeros(s) for s in shapes], meta["rank"], meta["mcr"], meta["iters"], meta["start"])
        assert np.array_equal(st.codec.p_flat.numpy(), want[f"rank{w}_p0"])
        states.append(st)
    res = [[torch.zeros(s) for s in shapes] for _ in range(world)]
    worst = 0.0
    for t in range(meta["steps"]):
        grads = [scenario_inputs(meta, t, res[w], w) for w in range(world)]
        outs = MW.run_workers(states, grads)
        for w in range(world):
            for i in range(len(shapes)):
                for got, k in ((outs[w][i], f"rank{w}_s{t}_out_{i}"), (grads[w][i], f"rank{w}_s{t}_res_{i}")):
                    ref = torch.from_numpy(want[k])
                    if world == 2:  # a + b == b + a: the rank-order sum is the ring's, bitwise
                        assert torch.equal(got, ref), (k, float((got - ref).abs().max()))
                    worst = max(worst, float((got - ref).norm()) / max(float(ref.norm()), 1e-30))
        res = grads
    assert worst < 1e-5, worst  # W = 4: gloo sums in another order (rounding only)


def _pipeline_worker(rank, world, initfile, corrupt, q, dtype="f32"):
    torch.distributed.init_process_group("gloo", init_method=f"file://{initfile}", rank=rank, world_size=world)
    torch.set_num_threads(1)
    try:
        c = dict(shapes=[(48, 32), (48, 32), (64, 8, 3, 3), (16,), (100, 20)], rank=2, iters=2, mcr=2,
                 dtype=dtype)
        st = O.policy_init([torch.zeros(s) for s in c["shapes"]], c["rank"], c["mcr"], c["iters"], 0)
        for buf in (st.codec.p_flat, st.codec.q_flat):  # one common injected state
            torch.distributed.broadcast(buf, src=0)

        def step(grads):  # the reference restatement over the real gloo all-reduce
            g32 = [g.float() for g in grads]  # bf16: the device path's fp32 arithmetic on bf16 storage
            outs = O.policy_step(st, g32, world, lambda b: torch.distributed.all_reduce(b))
            for g, r in zip(grads, g32):
                if g is not r:
                    g.copy_(r)  # the residual, stored in bf16
            if corrupt and rank == 1:
                outs[2] = outs[2] + (5e-2 if dtype == "bf16" else 1e-3)  # above each dtype's bound
            return outs

        p0, q0 = st.codec.p_flat.clone(), st.codec.q_flat.clone()
        dt = torch.bfloat16 if dtype == "bf16" else torch.float32
        outs, ress, errs = bench.parity_collect(step, c["shapes"], world, rank, "gloo", torch.device("cpu"), dt)
        if rank == 0:
            q.put(bench.parity_check(c, world, p0, q0, outs, ress) | {"errs": errs})
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.parametrize("corrupt", [False, True])
def test_gather_and_oracle_pipeline_gloo(corrupt):
    ctx = torch.multiprocessing.get_context("spawn")
    q = ctx.SimpleQueue()
    with tempfile.TemporaryDirectory() as td:
        torch.multiprocessing.spawn(_pipeline_worker, args=(2, os.path.join(td, "init"), corrupt, q),
                                    nprocs=2, join=True)
    r = q.get()
    assert r["errs"] == [None, None]
    if corrupt:
        assert not r["ok"] and r["steps"][0]["max_rel_out"] > 1e-5
        assert not r["outputs_equal_on_all_ranks"]
    else:
        assert r["ok"] and r["outputs_equal_on_all_ranks"], r
        assert all(s["max_rel_out"] == 0.0 and s["max_rel_res"] == 0.0 for s in r["steps"]), r


@pytest.mark.parametrize("corrupt", [False, True])
def test_gather_and_oracle_pipeline_gloo_bf16(corrupt):
    """bf16 gradients (cfg4's dtype): rank 0 rebuilds every worker's input from its gathered
    bf16 residual, so the oracle sees exactly the values the step saw; the outputs match
    bitwise, the bf16-stored residuals within bf16 rounding, and a corrupted rank is caught."""
    ctx = torch.multiprocessing.get_context("spawn")
    q = ctx.SimpleQueue()
    with tempfile.TemporaryDirectory() as td:
        torch.multiprocessing.spawn(_pipeline_worker, args=(2, os.path.join(td, "init"), corrupt, q, "bf16"),
                                    nprocs=2, join=True)
    r = q.get()
    assert r["errs"] == [None, None]
    if corrupt:
        assert not r["ok"]
    else:
        assert r["ok"] and r["outputs_equal_on_all_ranks"], r
        assert all(s["max_rel_out"] == 0.0 and s["max_rel_res"] <= 4e-3 for s in r["steps"]), r
