"""Host-memory end-to-end rate (north_star: gradients arrive from a CPU-run model and the
decompressed gradients + residuals return to it), through powersgd_amd.host.HostPowerSGD.

One step = HostPowerSGD.aggregate on CPU gradients: pinned H2D of the compressed tensors,
the codec on the GPU, D2H of outputs and residuals, pipelined in bins over three streams
(uncompressed tensors stay on the host). Reported next to the device-resident rate and the
raw PCIe rates; this is NOT bench.py's `value`.

Also: the same with residual="device" (outputs-only D2H, the opt-in semantic variant), and the
raw PCIe rates one direction at a time and both directions at once on two streams (duplex).

usage: python tools/host_e2e.py [config] [steps] [chunks,...]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from powersgd_amd import Config, PowerSGD  # noqa: E402
from powersgd_amd.host import HostPowerSGD  # noqa: E402
from powersgd_amd.workloads import CONFIGS  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2_resnet50_r1"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    chunk_list = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1,2,4").split(",")]
    c = CONFIGS[cfg]
    dtype = torch.bfloat16 if c["dtype"] == "bf16" else torch.float32
    nbytes = sum(torch.Size(s).numel() for s in c["shapes"]) * (2 if dtype == torch.bfloat16 else 4)
    res = {"workload": cfg, "gradient_bytes": nbytes, "host_e2e": {}}
    for mode in ("host", "device"):
        for chunks in chunk_list:
            params = [torch.zeros(s, dtype=dtype) for s in c["shapes"]]
            host = HostPowerSGD(params, Config(c["rank"], c["mcr"], c["iters"], 0), devices=[0], chunks=chunks,
                                residual=mode)
            host.pin_gradients(params)
            for p in params:
                p.grad.normal_()
            grads = [p.grad for p in params]
            for _ in range(3):
                host.aggregate(grads)
            t0 = time.perf_counter()
            for _ in range(steps):
                host.aggregate(grads)
            e2e = (time.perf_counter() - t0) / steps
            key = f"chunks{chunks}" + ("" if mode == "host" else "_device_residual")
            res["host_e2e"][key] = {"ms": round(e2e * 1e3, 3), "GBs": round(nbytes / e2e / 1e9, 2)}
            del host, params, grads

    dev = torch.device("cuda:0")
    psgd = PowerSGD([torch.zeros(s, device=dev, dtype=dtype) for s in c["shapes"]],
                    Config(c["rank"], c["mcr"], c["iters"], 0))
    dg = [torch.randn(s, device=dev).to(dtype) for s in c["shapes"]]
    for _ in range(3):
        psgd.aggregate(dg)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        psgd.aggregate(dg)
    torch.cuda.synchronize()
    dev_t = (time.perf_counter() - t0) / steps
    res["device_resident"] = {"ms": round(dev_t * 1e3, 4), "GBs": round(nbytes / dev_t / 1e9, 1)}

    hb = torch.empty(16 << 20, dtype=torch.float32).pin_memory()
    db = torch.empty_like(hb, device=dev)
    rates = {}
    for name, fn in (("h2d", lambda: db.copy_(hb, non_blocking=True)), ("d2h", lambda: hb.copy_(db, non_blocking=True))):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        rates[name] = round(10 * hb.numel() * 4 / (time.perf_counter() - t0) / 1e9, 1)
    # both directions at once, one stream each (PCIe is full duplex; do the DMA engines overlap?)
    hb2 = torch.empty_like(hb).pin_memory()
    db2 = torch.empty_like(db)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        with torch.cuda.stream(s1):
            db.copy_(hb, non_blocking=True)
        with torch.cuda.stream(s2):
            hb2.copy_(db2, non_blocking=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    rates["duplex_total"] = round(2 * 10 * hb.numel() * 4 / dt / 1e9, 1)
    rates["duplex_ms_per_pair"] = round(dt / 10 * 1e3, 3)
    rates["serial_ms_per_pair"] = round(hb.numel() * 4 / 1e9 * (1 / rates["h2d"] + 1 / rates["d2h"]) * 1e3, 3)
    res["pcie_GBs"] = rates
    res["pcie_bytes_per_step"] = "compressed gradients in + outputs and residuals out (uncompressed stay on host)"
    print(json.dumps(res))


if __name__ == "__main__":
    main()
