"""Does the step's context slow the even product? Runs PowerSGD.aggregate over rotating cold
gradient sets with an optional GPU spin (torch.cuda._sleep) between steps, so that whatever
the previous step's final pass left in flight (write-back of its 204 MB of stores) has drained
before the next step's k_even starts. Run under rocprofv3 --kernel-trace and compare k_even.
usage: python tools/even_context.py <config> <sleep_cycles> [steps]"""
import sys

import torch

sys.path.insert(0, ".")
from powersgd_amd import Config, PowerSGD  # noqa: E402
from powersgd_amd.workloads import CONFIGS  # noqa: E402

cfg, cycles = sys.argv[1], int(sys.argv[2])
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
c = CONFIGS[cfg]
dev = torch.device("cuda:0")
dtype = torch.bfloat16 if c["dtype"] == "bf16" else torch.float32
gen = torch.Generator(device=dev).manual_seed(1234)
sets = [[torch.randn(s, generator=gen, device=dev).to(dtype) for s in c["shapes"]] for _ in range(4)]
psgd = PowerSGD([torch.zeros(s, device=dev, dtype=dtype) for s in c["shapes"]], Config(c["rank"], c["mcr"], c["iters"], 0))
for k in range(steps):
    if cycles:
        torch.cuda._sleep(cycles)
    psgd.aggregate(sets[k % 4])
torch.cuda.synchronize()
print("done")
