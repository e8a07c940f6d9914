"""Cost of the DDP communication hook (powersgd_amd.ddp) against the reference flow
(optimizer_step) and plain DDP, on ONE GPU through a 1-rank RCCL group (the multi-GPU code path;
no xGMI traffic). The "model" holds the ResNet-50 parameter shapes; its loss is sum_i <p_i, x_i>
with fixed random x_i, so backward costs one elementwise pass and the gradients are x_i.

Per training iteration (forward + backward + gradient aggregation + SGD step), ms:
  ddp_allreduce    DDP with its default bucketed all-reduce (uncompressed)
  ddp_powersgd     DDP + powersgd_hook (buckets deferred to the last one, one aggregate)
  optimizer_step   no DDP: backward, then powersgd_amd.optimizer_step (the reference flow)
usage: python tools/ddp_cost.py [steps] [config]"""
import json
import os
import socket
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from powersgd_amd import Config, PowerSGD, optimizer_step  # noqa: E402
from powersgd_amd.ddp import PowerSGDState, powersgd_hook  # noqa: E402
from powersgd_amd.workloads import CONFIGS  # noqa: E402


class Model(torch.nn.Module):
    def __init__(self, shapes, dev):
        super().__init__()
        self.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.zeros(s, device=dev)) for s in shapes])
        g = torch.Generator(device=dev).manual_seed(5)
        self.xs = [torch.randn(s, generator=g, device=dev) for s in shapes]

    def forward(self, z):  # z: a dummy input (DDP's forward needs one)
        return sum((p * x).sum() for p, x in zip(self.ps, self.xs)) + z.sum()


def timed(fn, steps):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    cfg = sys.argv[2] if len(sys.argv) > 2 else "cfg2_resnet50_r1"
    c = CONFIGS[cfg]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    torch.distributed.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                         device_id=dev)
    conf = Config(c["rank"], c["mcr"], c["iters"], 0)
    z = torch.zeros(1, device=dev)
    res = {"workload": cfg, "steps": steps, "note": "1-rank RCCL group on one GPU; ms per training iteration"}
    try:
        m = Model(c["shapes"], dev)
        ddp = torch.nn.parallel.DistributedDataParallel(m, device_ids=[0])
        opt = torch.optim.SGD(ddp.parameters(), lr=1e-3)

        def it_ddp():
            opt.zero_grad(set_to_none=True)
            ddp(z).backward()
            opt.step()
        res["ddp_allreduce"] = round(timed(it_ddp, steps), 4)

        m2 = Model(c["shapes"], dev)
        ddp2 = torch.nn.parallel.DistributedDataParallel(m2, device_ids=[0])
        state = PowerSGDState(conf, params=list(m2.parameters()))
        ddp2.register_comm_hook(state, powersgd_hook)
        opt2 = torch.optim.SGD(ddp2.parameters(), lr=1e-3)

        def it_hook():
            opt2.zero_grad(set_to_none=True)
            ddp2(z).backward()
            opt2.step()
        res["ddp_powersgd"] = round(timed(it_hook, steps), 4)

        m3 = Model(c["shapes"], dev)
        opt3 = torch.optim.SGD(m3.parameters(), lr=1e-3)
        agg = PowerSGD(list(m3.parameters()), conf)

        def it_ref():
            m3(z).backward()  # p.grad holds the residual: backward adds onto it (reference README)
            optimizer_step(opt3, agg)
        res["optimizer_step"] = round(timed(it_ref, steps), 4)

        def codec_only():
            agg.aggregate([p.grad for p in m3.parameters()])
        res["codec_only"] = round(timed(codec_only, steps), 4)
    finally:
        torch.distributed.destroy_process_group()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
