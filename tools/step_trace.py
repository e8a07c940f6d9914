"""Plain world-size-1 steps of one config (no timing events, no other blocks): run under
rocprofv3 --kernel-trace to see a step's kernel sequence and its launch gaps as the bench's
timed loop runs them. usage: python tools/step_trace.py <config> [steps] [rank override]
PSGD_TRACE_IDLE_US=<us>: an idle GPU spin of that length between steps (torch.cuda._sleep), so that
each step starts after the GPU idled (the memory system drained of in-flight requests).
PSGD_TRACE_FLUSH=1: a HIP event with the default (system-scope release) fence recorded after each
step, which writes the L2s' dirty lines back before the next step's first kernel starts."""
import os
import sys

import torch

sys.path.insert(0, ".")
from powersgd_amd import Config, PowerSGD  # noqa: E402
from powersgd_amd.workloads import CONFIGS  # noqa: E402

cfg = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
dev = torch.device("cuda:0")
c = dict(CONFIGS[cfg])
if len(sys.argv) > 3:
    c["rank"] = int(sys.argv[3])
dtype = torch.bfloat16 if c["dtype"] == "bf16" else torch.float32
gen = torch.Generator(device=dev).manual_seed(1)
sets = [[torch.randn(s, generator=gen, device=dev).to(dtype) for s in c["shapes"]] for _ in range(4)]
psgd = PowerSGD([torch.zeros(s, device=dev, dtype=dtype) for s in c["shapes"]], Config(c["rank"], c["mcr"], c["iters"], 0))
idle = float(os.environ.get("PSGD_TRACE_IDLE_US", "0"))
flush = os.environ.get("PSGD_TRACE_FLUSH") == "1"
for k in range(steps):
    if idle > 0:
        torch.cuda._sleep(int(idle * 2100))  # ~2.1 GHz shader clock under load
    psgd.aggregate(sets[k % 4])
    if flush:
        torch.cuda.Event().record()
torch.cuda.synchronize()
print("done")
