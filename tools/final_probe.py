"""Final-pass rate per matrix geometry (diagnostic tool): single-shape workloads of ~100 MB,
rank 1 / 4, I = 2, timed with the library's own final-pass events.
usage: python tools/final_probe.py [rank ...]"""
import sys

import torch

from powersgd_amd import Config, PowerSGD

SETS = {
    "one (49152,512)": [(49152, 512)],
    "one (5120,4608)": [(5120, 4608)],
    "m147  (4096,147)x42": [(4096, 147)] * 42,
    "m256  (1024,256)x96": [(1024, 256, 1, 1)] * 96,
    "m512  (2048,512)x24": [(2048, 512, 1, 1)] * 24,
    "m576  (4096,576)x10": [(4096, 64, 3, 3)] * 10,
    "m1024 (256,1024)x96": [(256, 1024, 1, 1)] * 96,
    "m2048 (512,2048)x24": [(512, 2048, 1, 1)] * 24,
    "m2304 (256,2304)x40": [(256, 256, 3, 3)] * 40,
    "m4608 (512,4608)x10": [(512, 512, 3, 3)] * 10,
}


def main():
    ranks = [int(x) for x in sys.argv[1:]] or [1]
    dev = torch.device("cuda", 0)
    for r in ranks:
        for name, shapes in SETS.items():
            gen = torch.Generator(device=dev).manual_seed(1)
            grads = [torch.randn(s, generator=gen, device=dev) for s in shapes]
            params = [torch.zeros(s, device=dev) for s in shapes]
            psgd = PowerSGD(params, Config(r, 2, 2, 0))
            plan = psgd._powersgd._plan
            for _ in range(5):
                psgd.aggregate(grads)
            torch.cuda.synchronize()
            plan.set_timing(True)
            for _ in range(30):
                psgd.aggregate(grads)
            torch.cuda.synchronize()
            ms, n = plan.timing_read()
            plan.set_timing(False)
            us = ms / max(n, 1) * 1e3
            nb = sum(g.numel() for g in grads) * 4
            fused = plan.fused_final(psgd._powersgd.step_counter - 1)
            print(f"r{r} {name:22s} fused={fused} final {us:7.2f} us  {3 * nb / us / 1e3:6.0f} GB/s (r1w2 bytes)",
                  flush=True)
            del psgd, grads, params
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
