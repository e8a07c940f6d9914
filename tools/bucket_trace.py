"""A few plain cfg2 steps through the library's RCCL path on a 1-rank RCCL group (the W > 1 code
path on one GPU), for a kernel + HIP API trace of the bucketed overlap (PSGD_COMM_BUCKETS=2)
against the single-collective step. Run under rocprofv3; prints the mean ms per step.
usage: rocprofv3 --kernel-trace --hip-runtime-trace ... -- python3 tools/bucket_trace.py [steps]
(round 5 traced PSGD_COMM_BUCKETS=2 with it, profiles/r05/bucket_trace; that mode is removed since)"""
import os
import socket
import sys
import time

import torch

sys.path.insert(0, ".")
from powersgd_amd import Config, PowerSGD  # noqa: E402
from powersgd_amd.workloads import CONFIGS  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
cfg = os.environ.get("TRACE_CFG", "cfg2_resnet50_r1")
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
with socket.socket() as sk:
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
torch.distributed.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                     device_id=dev)
c = CONFIGS[cfg]
gen = torch.Generator(device=dev).manual_seed(5)
sets = [[torch.randn(s, generator=gen, device=dev) for s in c["shapes"]] for _ in range(4)]
psgd = PowerSGD([torch.zeros(s, device=dev) for s in c["shapes"]], Config(c["rank"], c["mcr"], c["iters"], 0))
for k in range(10):
    psgd.aggregate(sets[k % 4])
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(steps):
    psgd.aggregate(sets[k % 4])
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / steps * 1e3
print(f"{cfg} buckets={os.environ.get('PSGD_COMM_BUCKETS', '1')} ms/step {dt:.4f}")
torch.distributed.destroy_process_group()
