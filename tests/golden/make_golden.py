"""Generate golden fixtures by running the REFERENCE (epfml/powersgd) on CPU.

Run in the dev container only (the reference is not on the GPU box):

    PYTHONPATH=/root/reference python tests/golden/make_golden.py

Writes small ``.npz`` fixtures (no pickles) + ``manifest.json`` into this
directory. Fixtures are data only: inputs, the reference's initial P/Q state,
and the reference's outputs / residuals / post-step state. They pin
``oracle/powersgd_oracle.py`` (tests/test_oracle_golden.py), which in turn is
the checker for the HIP path.

F1  small shapes, every branch (rank 1 joint norm, rank cap, 1x1 conv mask
    quirk, 1-D tensors compressed, zero gradients, warm-up, alternation,
    fp64 default dtype), 3-4 steps with error feedback.
F2  the F1 shape set at world size 2 and 4 over gloo (per-rank inputs).
F3  BASELINE configs at full size, checksums only, P0/Q0 injected from the
    portable hash generator.
F4  cfg4 with bf16-rounded inputs upcast to fp32 (the reference rejects bf16).
"""
from __future__ import annotations

import json
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
if "/root/reference" not in sys.path:
    sys.path.insert(0, "/root/reference")

from powersgd_amd.workloads import CONFIGS, hash_normal, hash_tensors  # noqa: E402

SMALL_A = [
    (16, 8, 3, 3), (16, 8, 3, 3), (16, 8, 3, 3),  # one shape group, B=3 (rank-1 joint norm)
    (3, 200),            # r capped at 3 when rank=4
    (64, 16, 1, 1),      # 1x1 conv: mask uses min(shape)=1
    (16,), (64,),        # 1-D (compressed only at very low min_compression_rate)
    (8, 16), (32, 8),
    (37, 53),            # odd sizes (no 16-byte vector path)
    (120, 40),
]

# name -> (shapes, rank, mcr, iters, start_after, steps, dtype, zero_at)
SCENARIOS = {
    "refmodel_r1_i1_warmup1": (None, 1, 10, 1, 1, 2, "f32", None),
    "refmodel_r2_i3_mcr10_f64": (None, 2, 10, 3, 0, 1, "f64", None),
    "refmodel_r2_i3_mcr10": (None, 2, 10, 3, 0, 2, "f32", None),
    "small_r1_i2": (SMALL_A, 1, 2, 2, 0, 3, "f32", None),
    "small_r2_i1": (SMALL_A, 2, 2, 1, 0, 4, "f32", None),
    "small_r4_i2_mcr0.1": (SMALL_A, 4, 0.1, 2, 0, 3, "f32", None),
    "small_r4_i3": (SMALL_A, 4, 1.0, 3, 1, 4, "f32", None),
    "small_r1_i4": (SMALL_A, 1, 2, 4, 0, 3, "f32", None),
    "small_r2_i2_zero": (SMALL_A, 2, 2, 2, 0, 3, "f32", (1, [0, 3, 9])),
    "small_r1_i2_zero": (SMALL_A, 1, 2, 2, 0, 3, "f32", (1, [0, 1, 2, 9])),
}
MULTI = {"small_r1_i2": (2, 4), "small_r4_i2_mcr0.1": (2,), "small_r2_i1": (2,)}


def refmodel_shapes():
    torch.manual_seed(0)
    m = torch.nn.Sequential(
        torch.nn.Conv2d(3, 100, 3), torch.nn.ReLU(), torch.nn.Conv2d(100, 50, 5), torch.nn.Linear(50, 1)
    )
    return [tuple(p.shape) for p in m.parameters()]


def run_scenario(name, rank_id=0, world=1):
    import powersgd
    from powersgd import Config, PowerSGD

    shapes, rank, mcr, iters, start, steps, dt, zero_at = SCENARIOS[name]
    if shapes is None:
        shapes = refmodel_shapes()
    dtype = torch.float64 if dt == "f64" else torch.float32
    prev = torch.get_default_dtype()
    torch.set_default_dtype(dtype)
    try:
        params = [torch.zeros(s, dtype=dtype) for s in shapes]
        psgd = PowerSGD(params, Config(rank, mcr, iters, start))
        rec = {
            "mask": np.array(psgd.is_compressed_mask, dtype=np.bool_),
            "p0": psgd._powersgd._ps_buffer.numpy().copy(),
            "q0": psgd._powersgd._qs_buffer.numpy().copy(),
            "compression_rate": np.array(psgd._powersgd.compression_rate),
        }
        grads = [torch.zeros(s, dtype=dtype) for s in shapes]
        for t in range(steps):
            fresh = hash_tensors(shapes, seed=1000 + t + 100 * rank_id)
            for i, (g, f) in enumerate(zip(grads, fresh)):
                g.add_(torch.from_numpy(f).to(dtype))  # error feedback: residual + new grad
                if zero_at is not None and zero_at[0] == t and i in zero_at[1]:
                    g.zero_()
            # inputs are not stored: step t's input = step t-1's residual + hash_tensors(1000+t)
            outs = psgd.aggregate(grads)
            for i in range(len(shapes)):
                rec[f"s{t}_out_{i}"] = outs[i].detach().clone().numpy()
                rec[f"s{t}_res_{i}"] = grads[i].clone().numpy()
            rec[f"s{t}_p"] = psgd._powersgd._ps_buffer.numpy().copy()
            rec[f"s{t}_q"] = psgd._powersgd._qs_buffer.numpy().copy()
            rec[f"s{t}_step"] = np.array([psgd.step_counter, psgd._powersgd.step_counter])
    finally:
        torch.set_default_dtype(prev)
    meta = dict(shapes=[list(s) for s in shapes], rank=rank, mcr=mcr, iters=iters, start=start,
                steps=steps, dtype=dt, zero_at=zero_at, world=world)
    return rec, meta


def _worker(rank_id, world, name, initfile, outdir):
    torch.distributed.init_process_group("gloo", init_method=f"file://{initfile}", rank=rank_id,
                                         world_size=world)
    torch.set_num_threads(1)
    rec, _ = run_scenario(name, rank_id, world)
    np.savez_compressed(os.path.join(outdir, f"r{rank_id}.npz"), **rec)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def run_multi(name, world):
    with tempfile.TemporaryDirectory() as td:
        initfile = os.path.join(td, "init")
        torch.multiprocessing.spawn(_worker, args=(world, name, initfile, td), nprocs=world, join=True)
        merged = {}
        for r in range(world):
            with np.load(os.path.join(td, f"r{r}.npz")) as z:
                for k in z.files:
                    merged[f"rank{r}_{k}"] = z[k]
    return merged


def checksums(arr: np.ndarray, nsamp: int = 256):
    a = arr.astype(np.float64).reshape(-1)
    idx = np.linspace(0, a.size - 1, num=min(nsamp, a.size)).astype(np.int64)
    return a.sum(), np.sqrt((a * a).sum()), a[idx]


def run_config(cfg_name, steps):
    from powersgd import Config, PowerSGD

    c = CONFIGS[cfg_name]
    shapes = c["shapes"]
    params = [torch.zeros(s) for s in shapes]
    psgd = PowerSGD(params, Config(c["rank"], c["mcr"], c["iters"], 0))
    ps, qs = psgd._powersgd._ps_buffer, psgd._powersgd._qs_buffer
    ps.copy_(torch.from_numpy(hash_normal(7, ps.numel(), stream=1)))
    qs.copy_(torch.from_numpy(hash_normal(7, qs.numel(), stream=2)))
    rec = {"mask": np.array(psgd.is_compressed_mask), "p0_sum": np.array(ps.double().sum().item())}
    grads = [torch.zeros(s) for s in shapes]
    for t in range(steps):
        fresh = hash_tensors(shapes, seed=2000 + t)
        for g, f in zip(grads, fresh):
            ft = torch.from_numpy(f)
            if c["dtype"] == "bf16":
                ft = ft.to(torch.bfloat16).float()
            g.add_(ft)
            if c["dtype"] == "bf16":  # the residual is stored in bf16 in the bf16 workload
                g.copy_(g.to(torch.bfloat16).float())
        outs = psgd.aggregate(grads)
        sums = np.zeros((len(shapes), 4))
        samples = []
        for i in range(len(shapes)):
            so, no, xo = checksums(outs[i].numpy())
            sr, nr, xr = checksums(grads[i].numpy())
            sums[i] = (so, no, sr, nr)
            samples.append(np.stack([xo, xr]) if xo.size == 256 else np.zeros((2, 256)))
        rec[f"s{t}_sums"] = sums
        rec[f"s{t}_samples"] = np.stack(samples)
        rec[f"s{t}_p_sum"] = np.array(ps.double().sum().item())
        rec[f"s{t}_q_sum"] = np.array(qs.double().sum().item())
    return rec


def main():
    manifest = {"scenarios": {}, "multi": {}, "configs": {}}
    for name in SCENARIOS:
        rec, meta = run_scenario(name)
        np.savez_compressed(os.path.join(HERE, f"F1_{name}.npz"), **rec)
        manifest["scenarios"][name] = meta
        print("F1", name, flush=True)
    for name, worlds in MULTI.items():
        for w in worlds:
            rec = run_multi(name, w)
            np.savez_compressed(os.path.join(HERE, f"F2_{name}_w{w}.npz"), **rec)
            manifest["multi"][f"{name}_w{w}"] = dict(scenario=name, world=w)
            print("F2", name, w, flush=True)
    torch.set_num_threads(8)
    for cfg, steps in (("cfg1_1024sq_r1", 2), ("cfg2_resnet50_r1", 2), ("cfg3_resnet50_r4", 2),
                       ("cfg5_lstm_r1_i4", 3), ("cfg4_llama_r2_bf16", 1)):
        rec = run_config(cfg, steps)
        tag = "F4" if cfg.startswith("cfg4") else "F3"
        np.savez_compressed(os.path.join(HERE, f"{tag}_{cfg}.npz"), **rec)
        manifest["configs"][cfg] = dict(steps=steps, p0_seed=7, grad_seed=2000, tag=tag)
        print(tag, cfg, flush=True)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
