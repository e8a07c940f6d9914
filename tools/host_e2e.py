"""Host-memory end-to-end rate (north_star: gradients arrive from a CPU-run model and the
decompressed gradients + residuals return to it).

One step = pinned H2D of every gradient tensor -> PowerSGD.aggregate on the GPU -> D2H of
every output and of every residual (error-feedback buffer) into pinned host memory.
Reported next to the device-resident rate; this is NOT bench.py's `value`.

usage: python tools/host_e2e.py [config] [steps]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from powersgd_amd import Config, PowerSGD  # noqa: E402
from powersgd_amd.workloads import CONFIGS  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2_resnet50_r1"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    c = CONFIGS[cfg]
    dtype = torch.bfloat16 if c["dtype"] == "bf16" else torch.float32
    dev = torch.device("cuda:0")
    host_g = [torch.randn(s).to(dtype).pin_memory() for s in c["shapes"]]
    host_out = [torch.empty(s, dtype=dtype).pin_memory() for s in c["shapes"]]
    host_res = [torch.empty(s, dtype=dtype).pin_memory() for s in c["shapes"]]
    dev_g = [torch.empty(s, dtype=dtype, device=dev) for s in c["shapes"]]
    psgd = PowerSGD([torch.zeros(s, device=dev, dtype=dtype) for s in c["shapes"]],
                    Config(c["rank"], c["mcr"], c["iters"], 0))
    nbytes = sum(t.numel() * t.element_size() for t in host_g)

    def step():
        for d, h in zip(dev_g, host_g):
            d.copy_(h, non_blocking=True)
        outs = psgd.aggregate(dev_g)
        for h, o in zip(host_out, outs):
            h.copy_(o, non_blocking=True)
        for h, d in zip(host_res, dev_g):
            h.copy_(d, non_blocking=True)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    e2e = (time.perf_counter() - t0) / steps

    for _ in range(3):
        psgd.aggregate(dev_g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        psgd.aggregate(dev_g)
    torch.cuda.synchronize()
    dev_t = (time.perf_counter() - t0) / steps

    # raw PCIe rates for context (one 64 MiB pinned buffer each way)
    hb = torch.empty(16 << 20, dtype=torch.float32).pin_memory()
    db = torch.empty_like(hb, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        db.copy_(hb, non_blocking=True)
    torch.cuda.synchronize()
    h2d = 10 * hb.numel() * 4 / (time.perf_counter() - t0) / 1e9
    t0 = time.perf_counter()
    for _ in range(10):
        hb.copy_(db, non_blocking=True)
    torch.cuda.synchronize()
    d2h = 10 * hb.numel() * 4 / (time.perf_counter() - t0) / 1e9
    print(json.dumps({
        "workload": cfg, "gradient_bytes": nbytes,
        "end_to_end_ms": round(e2e * 1e3, 3), "end_to_end_GBs": round(nbytes / e2e / 1e9, 2),
        "device_resident_ms": round(dev_t * 1e3, 4), "device_resident_GBs": round(nbytes / dev_t / 1e9, 1),
        "pcie_h2d_GBs": round(h2d, 1), "pcie_d2h_GBs": round(d2h, 1),
        "bytes_over_pcie_per_step": 3 * nbytes,
    }))


if __name__ == "__main__":
    main()
