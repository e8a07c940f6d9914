"""Benchmark of the PowerSGD hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config NAME]

One step = one ``PowerSGD.aggregate`` over the synthetic gradients of the workload
(compressed matrices: power iterations + factor all-reduce + fused residual/output
pass; uncompressed tensors: flat pack + all-reduce), inputs resident in HBM.
N > 1: one process per GPU (torch.distributed.run), every rank holds its own gradients
(data parallel, weak scaling) and the P/Q factors are SUM-all-reduced over RCCL.

Prints ONE JSON line on rank 0. ``value`` = gradient bytes processed by all ranks per
second (GB/s). ``roofline`` = the final pass, the dominant kernel: k_final_odd (the last
odd power iteration fused with the residual/output writes) or k_apply (residual + output
after an even last iteration), timed with HIP events on the launch stream over the timed
region.
``cpu_baseline`` = the CPU oracle (bit-identical restatement of the reference) on a
bounded sample, rank 0 at N = 1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from powersgd_amd import Config, PowerSGD  # noqa: E402
from powersgd_amd.workloads import CONFIGS  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="cfg2_resnet50_r1", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    return ap.parse_args()


def numel(s):
    n = 1
    for d in s:
        n *= d
    return n


def apply_alg_bytes(c, mask, world, fused):
    """Algorithmic HBM bytes of ONE final-pass launch + the factor panels it must read (fp32).
    k_apply: read G0, write residual, write output (s bytes each per element).
    k_final_odd (fused last odd iteration): read G0, write residual, and at world size 1
    write the output (2 or 3 s bytes per element). At world size 1 the same launch also
    packs the uncompressed tensors (read, write flat, write zero: 3 s bytes per element)."""
    s = 2 if c["dtype"] == "bf16" else 4
    terms = 1 if world == 1 else 2
    per = 3 if (not fused or world == 1) else 2
    total = 0
    for shp, comp in zip(c["shapes"], mask):
        if not comp:
            if world == 1:
                total += 3 * s * numel(shp)
            continue
        n = shp[0]
        m = numel(shp) // n
        r = min(c["rank"], n, m)
        total += per * s * n * m + 4 * terms * c["iters"] * r * (n + m)
    return total


def step_alg_bytes(c, mask, world, fused):
    """sum_c s*n*m*(I+3) + sum_c 4*I*r*(n+m) + sum_u 3*s*N. With the fused
    last odd iteration the gradient is read once less: (I+2) instead of (I+3)."""
    s = 2 if c["dtype"] == "bf16" else 4
    passes = c["iters"] + (2 if fused else 3)
    total = 0
    for shp, comp in zip(c["shapes"], mask):
        N = numel(shp)
        if comp:
            n = shp[0]
            m = N // n
            r = min(c["rank"], n, m)
            total += s * N * passes + 4 * c["iters"] * r * (n + m)
        else:
            total += 3 * s * N
    return total


def load_pmc_traffic(cfg):
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(cfg)
    except (OSError, ValueError):
        return None


def cpu_baseline(c, seconds):
    from oracle import powersgd_oracle as O

    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    cores = max(1, min(int(os.environ.get("OMP_NUM_THREADS", cores)), cores))
    torch.set_num_threads(cores)
    g = torch.Generator().manual_seed(0)
    shapes = c["shapes"]
    grads = [torch.randn(s, generator=g) for s in shapes]
    ps = O.policy_init([torch.zeros(s) for s in shapes], c["rank"], c["mcr"], c["iters"], 0)
    O.policy_step(ps, grads)  # warm-up
    times = []
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end or len(times) < 3:
        t0 = time.perf_counter()
        O.policy_step(ps, grads)
        times.append(time.perf_counter() - t0)
    s = 2 if c["dtype"] == "bf16" else 4
    byts = sum(numel(x) for x in shapes) * s
    t = statistics.median(times)
    return {"value": round(byts / t / 1e9, 4), "unit": "GB/s", "cores": cores, "kind": "port",
            "sample": f"{len(times)} oracle aggregate() steps of {c['name']} (fp32 CPU, median step "
                      f"{t*1e3:.1f} ms, {sum(times):.1f} s total)"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # rehearsal knobs for a one-GPU box (never set by the driver): every rank on cuda:0
        # over gloo exercises the N > 1 code path end to end; the real run is RCCL, one GPU
        # per rank
        if os.environ.get("PSGD_BENCH_ONE_DEVICE") == "1":
            local = 0
        torch.cuda.set_device(local)
        backend = os.environ.get("PSGD_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.distributed.init_process_group(backend)
    dev = torch.device("cuda", local)
    c = dict(CONFIGS[a.config])
    c["name"] = a.config
    dtype = torch.bfloat16 if c["dtype"] == "bf16" else torch.float32
    shapes = c["shapes"]

    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    grads = [torch.randn(s, generator=gen, device=dev, dtype=torch.float32).to(dtype) for s in shapes]
    params = [torch.zeros(s, device=dev, dtype=dtype) for s in shapes]
    psgd = PowerSGD(params, Config(c["rank"], c["mcr"], c["iters"], 0))
    codec = psgd._powersgd

    for _ in range(a.warmup):
        psgd.aggregate(grads)
    torch.cuda.synchronize()

    # timed region: K plain steps (no instrumentation inside)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        psgd.aggregate(grads)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    # roofline pass: the same K steps again with HIP events around every final-pass launch,
    # recorded by the library on the launch stream
    codec._plan.set_timing(True)
    for _ in range(a.steps):
        psgd.aggregate(grads)
    torch.cuda.synchronize()
    apply_total_ms, apply_launches = codec._plan.timing_read()
    codec._plan.set_timing(False)
    apply_ms = apply_total_ms / max(apply_launches, 1)
    timed_first = codec.step_counter - a.steps  # step indices of the instrumented pass

    s = 2 if dtype == torch.bfloat16 else 4
    grad_bytes = sum(numel(x) for x in shapes) * s
    ms_step = elapsed / a.steps * 1e3
    value = world * grad_bytes * a.steps / elapsed / 1e9
    mask = psgd.is_compressed_mask
    # which final pass each timed step took (I odd: steps alternate between the fused last odd
    # iteration and k_apply); bytes are averaged over the timed steps
    nf = sum(codec._plan.fused_final(t) for t in range(timed_first, codec.step_counter))
    frac_f = nf / a.steps
    ab = frac_f * apply_alg_bytes(c, mask, world, True) + (1 - frac_f) * apply_alg_bytes(c, mask, world, False)
    sb = frac_f * step_alg_bytes(c, mask, world, True) + (1 - frac_f) * step_alg_bytes(c, mask, world, False)
    kf = "k_final_odd (fused last odd iteration: product + residual" + (" + output)" if world == 1 else ")")
    kname = kf if nf == a.steps else "k_apply (fused residual + output)" if nf == 0 else f"{kf} / k_apply, alternating"
    achieved = ab / (apply_ms * 1e-3) / 1e9
    out = {
        "metric": "gradient GB/s compressed+decompressed (device-resident)",
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
        "data": "synthetic N(0,1) gradients of the named parameter shapes (torch.randn on device)",
        "config": {"workload": a.config, "rank": c["rank"], "num_iters_per_step": c["iters"],
                   "min_compression_rate": c["mcr"], "tensors": len(shapes),
                   "compressed_tensors": sum(mask), "gradient_bytes_per_rank": grad_bytes,
                   "parallelism": f"dp{world}"},
        "roofline": {"kernel": kname, "bound": "hbm",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": load_pmc_traffic(a.config),
                     "alg_bytes_per_launch": round(ab), "avg_launch_us": round(apply_ms * 1e3, 2)},
        "step_roofline": {"alg_bytes_per_step": round(sb),
                          "achieved_GBs": round(sb / (ms_step * 1e-3) / 1e9, 1),
                          "frac": round(sb / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(c, a.cpu_seconds)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
