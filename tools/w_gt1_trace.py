"""The world-size > 1 code path on ONE GPU: a 1-rank RCCL process group makes
is_distributed() True, so PowerSGD.aggregate runs the multi-GPU sequence (buckets, async
factor all-reduces, per-bucket kernels, write-only output pass). Run under rocprofv3
--kernel-trace to see that sequence. usage: python tools/w_gt1_trace.py <config> [steps]"""
import socket
import sys

import torch

sys.path.insert(0, ".")
from powersgd_amd import Config, PowerSGD  # noqa: E402
from powersgd_amd.workloads import CONFIGS  # noqa: E402

cfg = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
with socket.socket() as sk:
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
torch.distributed.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
c = CONFIGS[cfg]
dtype = torch.bfloat16 if c["dtype"] == "bf16" else torch.float32
gen = torch.Generator(device=dev).manual_seed(1)
sets = [[torch.randn(s, generator=gen, device=dev).to(dtype) for s in c["shapes"]] for _ in range(4)]
psgd = PowerSGD([torch.zeros(s, device=dev, dtype=dtype) for s in c["shapes"]], Config(c["rank"], c["mcr"], c["iters"], 0))
for k in range(steps):
    psgd.aggregate(sets[k % 4])
torch.cuda.synchronize()
torch.distributed.destroy_process_group()
print("done")
