"""Multi-worker parity on ONE GPU: W processes share cuda:0 and all-reduce the P/Q
factors (and the uncompressed flat buffer) with gloo. This runs the HIP path's world-
size > 1 code (phased compress -> all-reduce -> decompress, alpha = 1/W, uncompressed
tensors divided by W) against the reference's own gloo multi-worker goldens (F2)."""
import os
import tempfile

import numpy as np
import pytest
import torch

from golden_io import load, manifest, scenario_inputs
from parity_log import check

pytestmark = pytest.mark.gpu
MAN = manifest()
TOL_FREE = 1e-4


def _worker(rank_id, world, key, initfile):
    from powersgd_amd import Config, PowerSGD

    torch.distributed.init_process_group("gloo", init_method=f"file://{initfile}", rank=rank_id,
                                         world_size=world)
    try:
        info = MAN["multi"][key]
        meta = MAN["scenarios"][info["scenario"]]
        want = load("F2_" + key)
        pre = f"rank{rank_id}_"
        dev = torch.device("cuda:0")
        shapes = [tuple(s) for s in meta["shapes"]]
        psgd = PowerSGD([torch.zeros(s, device=dev) for s in shapes],
                        Config(meta["rank"], meta["mcr"], meta["iters"], meta["start"]))
        psgd._powersgd._ps_buffer.copy_(torch.from_numpy(want[pre + "p0"]).to(dev))
        psgd._powersgd._qs_buffer.copy_(torch.from_numpy(want[pre + "q0"]).to(dev))
        res = [torch.zeros(s) for s in shapes]
        for t in range(meta["steps"]):
            inputs = scenario_inputs(meta, t, res, rank_id)
            grads = [g.to(dev) for g in inputs]
            outs = psgd.aggregate(grads)
            torch.cuda.synchronize()
            for i, g in enumerate(inputs):
                scale = max(float(g.norm()), 1e-30)
                eo = float((outs[i].cpu() - torch.from_numpy(want[f"{pre}s{t}_out_{i}"])).norm()) / scale
                er = float((grads[i].cpu() - torch.from_numpy(want[f"{pre}s{t}_res_{i}"])).norm()) / scale
                check(eo, TOL_FREE, key, rank_id, t, i, "out")
                check(er, TOL_FREE, key, rank_id, t, i, "res")
            res = [g.cpu() for g in grads]
        torch.distributed.barrier()
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.parametrize("key", sorted(MAN["multi"]))
def test_multiworker_gloo_on_one_gpu(key):
    world = MAN["multi"][key]["world"]
    with tempfile.TemporaryDirectory() as td:
        torch.multiprocessing.spawn(_worker, args=(world, key, os.path.join(td, "init")), nprocs=world,
                                    join=True)


def _bucket_worker(rank_id, world, initfile, cfg, steps):
    """ResNet-50 shapes at world size `world`: the bucketed, overlapped collectives (default
    PSGD_BUCKETS = 4, async all-reduce per bucket slice) against the oracle run in the same
    processes over the same gloo group, and against the single-collective path. The even
    product's workgroup ranges are cut per bucket (k_even), so the two paths differ in which
    rows share a partial sum: equal to rounding, not bitwise."""
    import os as _os

    from oracle import powersgd_oracle as O
    from powersgd_amd import Config, PowerSGD
    from powersgd_amd.workloads import CONFIGS, hash_tensors

    torch.distributed.init_process_group("gloo", init_method=f"file://{initfile}", rank=rank_id,
                                         world_size=world)
    try:
        c = CONFIGS[cfg]
        shapes = c["shapes"]
        dev = torch.device("cuda:0")
        runs = []
        for buckets in ("4", "1"):
            _os.environ["PSGD_BUCKETS"] = buckets
            psgd = PowerSGD([torch.zeros(s, device=dev) for s in shapes], Config(c["rank"], c["mcr"], c["iters"], 0))
            ora = O.policy_init([torch.zeros(s) for s in shapes], c["rank"], c["mcr"], c["iters"], 0)
            ora.codec.p_flat.copy_(psgd._powersgd._ps_buffer.cpu())
            ora.codec.q_flat.copy_(psgd._powersgd._qs_buffer.cpu())
            res_d = [torch.zeros(s, device=dev) for s in shapes]
            res_c = [torch.zeros(s) for s in shapes]
            outs_all = []
            for t in range(steps):
                new = [torch.from_numpy(f) for f in hash_tensors(shapes, seed=500 + 10 * t + rank_id)]
                gd = [r + x.to(dev) for r, x in zip(res_d, new)]
                gc = [r + x for r, x in zip(res_c, new)]
                scale = [g.clone() for g in gc]
                od = psgd.aggregate(gd)
                oc = O.policy_step(ora, gc, world, lambda b: torch.distributed.all_reduce(b))
                torch.cuda.synchronize()
                for i, g in enumerate(scale):
                    tol = 1e-5 if t == 0 else TOL_FREE
                    check(_rel_err(od[i], oc[i], g), tol, cfg, buckets, rank_id, t, i, "out")
                    check(_rel_err(gd[i], gc[i], g), tol, cfg, buckets, rank_id, t, i, "res")
                outs_all.append([o.clone() for o in od] + [g.clone() for g in gd])
                res_d, res_c = gd, gc
            runs.append((len(psgd._powersgd._buckets), outs_all))
        assert runs[0][0] > 1 and runs[1][0] == 1, (runs[0][0], runs[1][0])
        for t, (a, b) in enumerate(zip(runs[0][1], runs[1][1])):
            for i, (x, y) in enumerate(zip(a, b)):
                check(_rel_err(x, y, y), 1e-5 if t == 0 else TOL_FREE, cfg, "buckets-vs-one", rank_id, t, i)
        torch.distributed.barrier()
    finally:
        _os.environ.pop("PSGD_BUCKETS", None)
        torch.distributed.destroy_process_group()


def _rel_err(a, b, scale):
    return float((a.double().cpu() - b.double().cpu()).norm()) / max(float(scale.double().norm()), 1e-30)


@pytest.mark.parametrize("cfg,world", [("cfg3_resnet50_r4", 2), ("cfg2_resnet50_r1", 2), ("cfg2_resnet50_r1", 4)])
def test_bucketed_collectives_vs_oracle(cfg, world):
    with tempfile.TemporaryDirectory() as td:
        torch.multiprocessing.spawn(_bucket_worker, args=(world, os.path.join(td, "init"), cfg, 2), nprocs=world,
                                    join=True)
