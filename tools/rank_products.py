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


# rank-k flops per element of the compressed matrices, per kernel family (x 2*r):
#   k_even: Gt X (iteration 0, no error-feedback term)                    -> 1
#   k_product_odd / k_odd_mfma: (G - P0 Q0t) X, error feedback on the fly -> 2
#   k_final_proj: P = G X, then residual / output = P Xt                  -> 2
#   k_final_odd: error feedback + product + reconstruction                 -> 3
#   k_apply: residual and output from I factors (I = 2)                    -> 2
FLOP_TERMS = {"psgd::k_even": 1, "psgd::k_product_odd": 2, "psgd::k_odd_mfma": 2,
              "psgd::k_final_proj": 2, "psgd::k_final_odd": 3, "psgd::k_apply": 2}
N_CU, N_SIMD, N_XCD = 256, 4, 8


def _pmc(d):
    acc = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").strip()
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: statistics.mean(v) for c, v in cs.items()} for k, cs in acc.items()}


def analyze(d, rank):
    """Per rank-k kernel: median us, GB/s of the gradient, TFLOP/s against the fp32 peak, and
    (when a PMC pass is present) MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x kernel cycles),
    kernel cycles = GRBM_GUI_ACTIVE / 8 (summed over the XCDs, MI355X_MICROARCH.md DVFS note),
    and VALU active = SQ_ACTIVE_INST_VALU x 4 (quad-cycles) / (SIMDs x kernel cycles)."""
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
    pmc = _pmc(d)
    for k, v in sorted(by.items()):
        fam = next((f for f in FLOP_TERMS if k.startswith(f)), None)
        if fam is None:
            continue
        us = statistics.median(v)
        flops = 2.0 * nmr * FLOP_TERMS[fam]
        tf = flops / (us * 1e-6) / 1e12
        gbs = 4.0 * nm / (us * 1e-6) / 1e9
        o = {"rank": rank, "kernel": k, "launches": len(v), "median_us": round(us, 2),
             "GBs_of_G": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 3),
             "TFLOPs": round(tf, 2), "fp32_peak_frac": round(tf / FP32_PEAK_TFLOPS, 4),
             "flop_per_byte": round(flops / (4.0 * nm), 2)}
        c = pmc.get(k)
        if c and c.get("GRBM_GUI_ACTIVE"):
            cyc = c["GRBM_GUI_ACTIVE"] / N_XCD
            simd_cyc = N_CU * N_SIMD * cyc
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                o["mfma_busy"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cyc, 4)
            if "SQ_ACTIVE_INST_VALU" in c:
                o["valu_active"] = round(4.0 * c["SQ_ACTIVE_INST_VALU"] / simd_cyc, 4)
            o["pmc_clock_GHz"] = round(cyc / (us * 1e3), 3)
        print(json.dumps(o))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]))
    else:
        analyze(sys.argv[2], int(sys.argv[3]))
