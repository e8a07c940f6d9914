"""Rank-k product kernels at ResNet-50 shapes: achieved TFLOP/s against the fp32 MFMA/VALU
peak and GB/s against HBM, per rank (the north star's "MFMA utilisation on the rank-k
matmuls").

usage (GPU box):
  python tools/rank_products.py run R            # 5 warm-up + 40 steps, prints ms/step
  rocprofv3 --kernel-trace -d DIR -o kt -- python3 tools/rank_products.py run R
  python tools/rank_products.py analyze DIR R     # per product kernel: us, GB/s, TFLOP/s

Algorithmic figures per product launch (all compressed matrices of the step):
bytes = s * sum(n*m) (+ factor panels, negligible); flops = 2*n*m*r*(1 + nres), where nres
is the number of earlier iterations whose error feedback the kernel forms on the fly
(iteration 0: 0, iteration 1: 1).
"""
import csv
import glob
import json
import os
import re
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: fp32 vector = fp32 matrix (no xf32 on gfx950)
HBM_PEAK_GBS = 8000.0


def _mats(rank):
    from powersgd_amd.workloads import resnet50_shapes
    out = []
    for s in resnet50_shapes():
        if len(s) < 2:
            continue
        n, m = s[0], 1
        for d in s[1:]:
            m *= d
        r = min(rank, n, m)
        if n * m / (0.5 * 2 * r * (n + m)) > 2:  # mcr = 2, I = 2 (powersgd.py:101-105, :292-294)
            out.append((n, m, r))
    return out


def run(rank):
    import time
    import torch
    from powersgd_amd import Config, PowerSGD
    from powersgd_amd.workloads import resnet50_shapes
    dev = torch.device("cuda:0")
    shapes = resnet50_shapes()
    gen = torch.Generator(device=dev).manual_seed(7)
    grads = [torch.randn(s, generator=gen, device=dev) for s in shapes]
    psgd = PowerSGD([torch.zeros(s, device=dev) for s in shapes], Config(rank, 2, 2, 0))
    for _ in range(5):
        psgd.aggregate(grads)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    K = 40
    for _ in range(K):
        psgd.aggregate(grads)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / K * 1e3
    gb = sum(g.numel() for g in grads) * 4 / (ms * 1e-3) / 1e9
    print(json.dumps({"rank": rank, "ms_per_step": round(ms, 4), "GBs": round(gb, 1)}))


def analyze(d, rank):
    mats = _mats(rank)
    nm = sum(n * m for n, m, _ in mats)
    nmr = sum(n * m * r for n, m, r in mats)
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(path)))
    by = defaultdict(list)
    for r in rows:
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").strip()
        by[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = []
    for k, v in sorted(by.items()):
        if not k.startswith(("psgd::k_product", "psgd::k_odd_mfma")):
            continue
        us = statistics.median(v)
        # even product = iteration 0 (no error-feedback terms); odd product = iteration 1
        even = k.startswith("psgd::k_product") and k.rstrip(">").split(",")[-1].strip() == "true"
        nres = 0 if even else 1
        flops = 2.0 * nmr * (1 + nres)
        tf = flops / (us * 1e-6) / 1e12
        gbs = 4.0 * nm / (us * 1e-6) / 1e9
        out.append({"rank": rank, "kernel": k, "launches": len(v), "median_us": round(us, 2),
                    "GBs": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 3),
                    "TFLOPs": round(tf, 2), "fp32_peak_frac": round(tf / FP32_PEAK_TFLOPS, 4),
                    "flop_per_byte": round(flops / (4.0 * nm), 2)})
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]))
    else:
        analyze(sys.argv[2], int(sys.argv[3]))
