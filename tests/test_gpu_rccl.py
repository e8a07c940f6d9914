"""The world-size > 1 step through the library's own RCCL communicator (psgd_aggregate_comm:
kernels and in-place SUM all-reduces on one stream, include/psgd.h) on ONE GPU: a 1-rank NCCL
process group makes is_distributed() True, so PowerSGD.aggregate takes exactly the code path
of an 8-GPU run (K-term final pass, write-only output pass, flat pack /W inside the last
collective). Checked per step against the CPU oracle (bit-identical to the reference) at
world size 1. Spawned in a child process so the process group does not leak into other tests."""
import os
import socket

import pytest
import torch

from parity_log import check

pytestmark = pytest.mark.gpu


def _rel(a, b, scale):
    return float((a.double().cpu() - b.double().cpu()).norm()) / max(float(scale.double().norm()), 1e-30)


def _worker(_, port, cfg, steps, env=None):
    os.environ.update(env or {})  # plan knobs, read at plan creation
    from oracle import powersgd_oracle as O
    from powersgd_amd import Config, PowerSGD, _lib
    from powersgd_amd.workloads import CONFIGS, hash_tensors

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    torch.distributed.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                         device_id=dev)
    try:
        c = CONFIGS[cfg]
        shapes = c["shapes"]
        dt = torch.bfloat16 if c["dtype"] == "bf16" else torch.float32
        psgd = PowerSGD([torch.zeros(s, device=dev, dtype=dt) for s in shapes],
                        Config(c["rank"], c["mcr"], c["iters"], 0))
        ora = O.policy_init([torch.zeros(s) for s in shapes], c["rank"], c["mcr"], c["iters"], 0)
        ora.codec.p_flat.copy_(psgd._powersgd._ps_buffer.cpu())
        ora.codec.q_flat.copy_(psgd._powersgd._qs_buffer.cpu())
        res_d = [torch.zeros(s, device=dev, dtype=dt) for s in shapes]
        res_c = [torch.zeros(s) for s in shapes]
        for t in range(steps):
            new = [torch.from_numpy(f) for f in hash_tensors(shapes, seed=900 + t)]
            gd = [(r.float() + x.to(dev)).to(dt) for r, x in zip(res_d, new)]
            # the oracle sees exactly the device inputs (bf16: the rounded values, upcast)
            gc = [g.float().cpu() for g in gd] if dt == torch.bfloat16 else [r + x for r, x in zip(res_c, new)]
            scale = [g.clone() for g in gc]
            od = psgd.aggregate(gd)
            oc = O.policy_step(ora, gc)
            torch.cuda.synchronize()
            assert isinstance(psgd._powersgd._comm, _lib.Comm)  # the library's RCCL path ran
            for i, g in enumerate(scale):
                tol = (1e-6 if c["rank"] == 1 else 1e-5) if t == 0 else 1e-4
                if dt == torch.bfloat16:
                    tol = 4e-3  # bf16 gradient storage; ~1.1e-3 RMS rounding
                check(_rel(od[i], oc[i], g), tol, cfg, t, i, "out")
                check(_rel(gd[i], gc[i], g), tol, cfg, t, i, "res")
            res_d, res_c = gd, gc
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.parametrize("cfg", ["cfg3_resnet50_r4", "cfg2_resnet50_r1", "cfg5_lstm_r1_i4", "cfg4_llama_r2_bf16"])
def test_rccl_step_one_rank_vs_oracle(cfg):
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    torch.multiprocessing.spawn(_worker, args=(port, cfg, 3), nprocs=1, join=True)


def test_rccl_kterm_own_row_blocks_vs_oracle():
    """The K-term final pass on its own row blocks (psgd_plan.cpp tiles_fin_kt, MatDesc::
    fin_rows_kt) at an odd block size, 5000 elements: ragged against every ResNet-50 row length,
    beside the projection form's default blocks of the same plan."""
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    torch.multiprocessing.spawn(_worker, args=(port, "cfg2_resnet50_r1", 2, {"PSGD_FIN_ELEMS_KT": "5000"}),
                                nprocs=1, join=True)
