"""The library's RCCL orchestration (psgd_aggregate_comm, psgd_plan.cpp) at world size W > 1 on ONE
GPU, through a stand-in collective library (tests/stubs/rccl_stub.hip, loaded with
PSGD_RCCL_LIB_FORCE): its communicator reports world W and its SUM all-reduce writes W x the
buffer, which is exactly the SUM over W ranks holding identical gradients. The result must match
W reference workers (oracle/multiworker.py: the CPU restatement, W threads meeting at the
reference's SUM all-reduce, powersgd.py:204-219; utils.py:43-47 for the flat tail) on identical
inputs. Unlike a 1-rank communicator (SUM = identity), this fails when the orchestration reduces
the wrong buffer, skips a collective, reduces twice, drops the flat tail, or passes the wrong
world size to the output pass — the negative controls below prove the test can fail.

Each case runs in a spawned child (its own environment, stub and process group)."""
import ctypes
import os
import socket

import pytest
import torch

from parity_log import check

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(REPO, "tests", "stubs", "librccl_stub.so")


# ranks 16 / 32 (the matrix-core even product and apply tiles, world size > 1: the output from
# the all-reduced factors): ragged strips, a narrow matrix, an m % 4 != 0 matrix, a flat tail
WIDE_SHAPES = [(300, 200), (64, 1000), (1000, 64), (96, 40), (333, 148), (200, 150), (40,), (130, 16, 3, 3)]
WIDE = {"wide16": {"shapes": WIDE_SHAPES, "rank": 16, "mcr": 0.1, "iters": 2, "dtype": "f32"},
        "wide32": {"shapes": WIDE_SHAPES, "rank": 32, "mcr": 0.1, "iters": 2, "dtype": "f32"},
        "wide16bf": {"shapes": WIDE_SHAPES, "rank": 16, "mcr": 0.1, "iters": 2, "dtype": "bf16"}}


def _spec(cfg):
    from powersgd_amd.workloads import CONFIGS
    return CONFIGS[cfg] if cfg in CONFIGS else WIDE[cfg]


def _port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _rel(a, b, scale):
    return float((a.double().cpu() - b.double().cpu()).norm()) / max(float(scale.double().norm()), 1e-30)


def _run(cfg, world, steps, port, env):
    """`steps` steps of cfg at world size `world` through the stub; returns per step the largest
    output / residual errors against W oracle workers and the stub's collective count."""
    os.environ["PSGD_RCCL_LIB_FORCE"] = STUB
    os.environ["PSGD_TESTING"] = "1"  # the override's second opt-in (psgd_comm.cpp)
    os.environ.update(env)
    from oracle import multiworker as MW
    from oracle import powersgd_oracle as O
    from powersgd_amd import Config, PowerSGD, _lib
    from powersgd_amd.workloads import hash_tensors

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    torch.distributed.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        stub = ctypes.CDLL(STUB)  # the same handle the library opened: one call counter
        stub.psgd_stub_calls.restype = ctypes.c_longlong
        c = _spec(cfg)
        shapes = c["shapes"]
        dt = torch.bfloat16 if c["dtype"] == "bf16" else torch.float32
        psgd = PowerSGD([torch.zeros(s, device=dev, dtype=dt) for s in shapes],
                        Config(c["rank"], c["mcr"], c["iters"], 0))
        codec = psgd._powersgd
        # the library's own communicator, created through the stand-in at world W (the process
        # group itself has one rank: it only makes is_distributed() true)
        codec._comm = _lib.Comm(world, 0, _lib.comm_unique_id(), 0)
        states = []
        for _ in range(world):
            st = O.policy_init([torch.zeros(s) for s in shapes], c["rank"], c["mcr"], c["iters"], 0)
            st.codec.p_flat.copy_(codec._ps_buffer.cpu())
            st.codec.q_flat.copy_(codec._qs_buffer.cpu())
            states.append(st)
        res_d = [torch.zeros(s, device=dev, dtype=dt) for s in shapes]
        res_c = [[torch.zeros(s) for s in shapes] for _ in range(world)]
        report = []
        for t in range(steps):
            new = [torch.from_numpy(f) for f in hash_tensors(shapes, seed=700 + t)]
            gd = [(r.float() + x.to(dev)).to(dt) for r, x in zip(res_d, new)]
            if dt == torch.bfloat16:  # the oracle sees exactly the device inputs (rounded, upcast)
                gc = [[g.float().cpu() for g in gd] for _ in range(world)]
            else:
                gc = [[r + x for r, x in zip(res_c[w], new)] for w in range(world)]
            scale = [g.clone() for g in gc[0]]
            n0 = stub.psgd_stub_calls()
            od = psgd.aggregate(gd)
            torch.cuda.synchronize()
            calls = stub.psgd_stub_calls() - n0
            want = MW.run_workers(states, gc)
            eo = max(_rel(od[i], want[0][i], scale[i]) for i in range(len(shapes)))
            er = max(_rel(gd[i], gc[0][i], scale[i]) for i in range(len(shapes)))
            report.append((eo, er, calls, sum(1 for m in psgd.is_compressed_mask if not m)))
            res_d, res_c = gd, gc
        return report
    finally:
        torch.distributed.destroy_process_group()


def _positive(_, port, cfg, world, steps):
    rep = _run(cfg, world, steps, port, {"PSGD_STUB_MODE": "sum"})
    c_iters = _spec(cfg)["iters"]
    for t, (eo, er, calls, nunc) in enumerate(rep):
        bf16 = _spec(cfg)["dtype"] == "bf16"
        tol = 4e-3 if bf16 else ((1e-5 if t == 0 else 1e-4))
        check(eo, tol, cfg, world, t, "out")
        check(er, tol, cfg, world, t, "res")
        # one collective per power iteration, plus the flat tail grouped with the last one (fp32
        # plans; a bf16 plan's uncompressed tensors are summed in their own dtype by the process
        # group, powersgd.py, not through the library's fp32 collective)
        assert calls == c_iters + (1 if nunc and not bf16 else 0), (cfg, calls)


@pytest.mark.parametrize("cfg,world", [("cfg2_resnet50_r1", 4), ("cfg3_resnet50_r4", 4),
                                       ("cfg5_lstm_r1_i4", 8), ("cfg4_llama_r2_bf16", 2),
                                       ("wide16", 2), ("wide32", 4), ("wide16bf", 2)])
def test_rccl_orchestration_world_w_vs_oracle(cfg, world):
    """psgd_aggregate_comm at world W, 2 steps, vs W reference workers."""
    torch.multiprocessing.spawn(_positive, args=(_port(), cfg, world, 2), nprocs=1, join=True)


def _negative(_, port, cfg, world, env, q):
    rep = _run(cfg, world, 1, port, env)
    q.put(max(rep[0][0], rep[0][1]))


@pytest.mark.parametrize("cfg,world,env", [
    ("cfg2_resnet50_r1", 4, {"PSGD_STUB_MODE": "twice"}),
    ("cfg2_resnet50_r1", 4, {"PSGD_STUB_MODE": "skip", "PSGD_STUB_SKIP_AT": "0"}),   # even Q
    ("cfg2_resnet50_r1", 4, {"PSGD_STUB_MODE": "skip", "PSGD_STUB_SKIP_AT": "1"}),   # odd P
    ("cfg2_resnet50_r1", 4, {"PSGD_STUB_MODE": "skip", "PSGD_STUB_SKIP_AT": "2"}),   # flat tail
    # cfg5: four collectives per step; a lost middle one (iteration 1's P) must show too
    ("cfg5_lstm_r1_i4", 8, {"PSGD_STUB_MODE": "skip", "PSGD_STUB_SKIP_AT": "1"}),
    ("cfg5_lstm_r1_i4", 8, {"PSGD_STUB_MODE": "twice"})],
    ids=["twice", "skip-q", "skip-p", "skip-flat", "cfg5-skip-p1", "cfg5-twice"])
def test_rccl_orchestration_negative_controls(cfg, world, env):
    """A collective library that reduces twice or drops one of the step's collectives must make
    the W-worker comparison fail (the positive test above is able to fail)."""
    ctx = torch.multiprocessing.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_negative, args=(0, _port(), cfg, world, env, q))
    p.start()
    err = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert err > 1e-2, (env, err)
