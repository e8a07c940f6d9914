"""One-shot all-reduce over IPC exchange buffers (psgd_aggregate_ipc, PSGD_COMM=ipc): W processes
on cuda:0, each mapping the others' exchange buffers with hipIpcOpenMemHandle. Every factor
all-reduce of a step (and the uncompressed tensors) is a device-side flag handshake plus a
rank-order sum, with no host barrier or synchronisation per step (gloo carries only the one-off
handle exchange). Checked against the reference's own multi-worker goldens (F2), like the
collective path; plus skewed ranks and the bounded wait."""
import gc
import os
import tempfile
import time

import pytest
import torch

from golden_io import load, manifest, scenario_inputs
from parity_log import check

pytestmark = pytest.mark.gpu
MAN = manifest()
TOL_FREE = 1e-4


def _worker(rank_id, world, key, initfile, skew, sessions=1, extra_steps=0, logfile=None):
    os.environ["PSGD_COMM"] = "ipc"
    torch.distributed.init_process_group("gloo", init_method=f"file://{initfile}", rank=rank_id, world_size=world)
    try:
        for n in range(sessions):
            _session(rank_id, world, key, skew, extra_steps, logfile, n)
            gc.collect()  # the codec is freed (its exchange region returns to the arena) before the next
    finally:
        torch.distributed.destroy_process_group()


def _log_session(psgd, rank_id, world, logfile, n):
    """Per session and peer: the region addresses, the nonce each peer announced and the nonce
    read through this process's mapping of it, and the process's arena counters."""
    import json

    plan = psgd._powersgd._plan
    own = plan.ipc_debug(rank_id)
    announced = [None] * world
    torch.distributed.all_gather_object(announced, own["own_nonce"])
    recs = []
    for w in range(world):
        d = plan.ipc_debug(w)
        recs.append({"session": n, "rank": rank_id, "peer": w, "own_va": hex(d["own_va"]), "peer_va": hex(d["peer_va"]),
                     "announced_nonce": announced[w], "nonce_seen": d["peer_nonce_seen"],
                     "arena": [d["arena_allocs"], d["arena_opens"], d["arena_reuses"], d["arena_frees"]]})
        assert d["peer_nonce_seen"] == announced[w], recs[-1]
    with open(logfile, "a") as f:
        for r in recs:
            f.write(json.dumps(r) + "\n")


def _session(rank_id, world, key, skew, extra_steps=0, logfile=None, n=0):
    from powersgd_amd import Config, PowerSGD

    info = MAN["multi"][key]
    meta = MAN["scenarios"][info["scenario"]]
    want = load("F2_" + key)
    pre = f"rank{rank_id}_"
    dev = torch.device("cuda:0")
    shapes = [tuple(s) for s in meta["shapes"]]
    psgd = PowerSGD([torch.zeros(s, device=dev) for s in shapes],
                    Config(meta["rank"], meta["mcr"], meta["iters"], meta["start"]))
    psgd._powersgd._ps_buffer.copy_(torch.from_numpy(want[pre + "p0"]).to(dev))
    psgd._powersgd._qs_buffer.copy_(torch.from_numpy(want[pre + "q0"]).to(dev))
    res = [torch.zeros(s) for s in shapes]
    for t in range(meta["steps"]):
        inputs = scenario_inputs(meta, t, res, rank_id)
        grads = [g.to(dev) for g in inputs]
        if skew and rank_id == t % world:
            time.sleep(0.3)  # this rank arrives late: the peers' kernels wait on its flags
        outs = psgd.aggregate(grads)
        torch.cuda.synchronize()
        for i, g in enumerate(inputs):
            scale = max(float(g.norm()), 1e-30)
            eo = float((outs[i].cpu() - torch.from_numpy(want[f"{pre}s{t}_out_{i}"])).norm()) / scale
            er = float((grads[i].cpu() - torch.from_numpy(want[f"{pre}s{t}_res_{i}"])).norm()) / scale
            check(eo, TOL_FREE, key, rank_id, t, i, "ipc-out")
            check(er, TOL_FREE, key, rank_id, t, i, "ipc-res")
        res = [g.cpu() for g in grads]
    assert psgd._powersgd._ipc_open
    if logfile:
        _log_session(psgd, rank_id, world, logfile, n)
    # more steps on random gradients: the session's flags reach epochs far above the next
    # session's first ones (the round-5 failing order: bench timing session, then a same-size
    # parity session in the same processes)
    gen = torch.Generator().manual_seed(100 + rank_id)
    for _ in range(extra_steps):
        psgd.aggregate([torch.randn(s, generator=gen).to(dev) for s in shapes])
    torch.cuda.synchronize()
    assert not psgd._powersgd.ipc_status(), "a device-side exchange wait timed out"
    psgd._powersgd.close_ipc()


@pytest.mark.parametrize("key", sorted(MAN["multi"]))
def test_ipc_one_shot_allreduce_matches_reference(key):
    world = MAN["multi"][key]["world"]
    with tempfile.TemporaryDirectory() as td:
        torch.multiprocessing.spawn(_worker, args=(world, key, os.path.join(td, "init"), False), nprocs=world,
                                    join=True)


def test_ipc_skewed_ranks():
    """One rank per step arrives 0.3 s late: the others' exchange kernels wait on its flag
    (device side) and the results still match the reference goldens."""
    key = sorted(k for k in MAN["multi"] if MAN["multi"][k]["world"] == 2)[0]
    with tempfile.TemporaryDirectory() as td:
        torch.multiprocessing.spawn(_worker, args=(2, key, os.path.join(td, "init"), True), nprocs=2, join=True)


def test_ipc_sessions_back_to_back():
    """Three codecs of the same shapes one after the other in the same processes, each freed
    before the next is made, each session first matched to the reference goldens step by step and
    then run 40 steps further (its flags end far above the next session's first epochs: the
    round-5 r05a-new order). The exchange arena makes the sessions share ONE region per process:
    per session and peer the test logs the region addresses, the nonce each peer announced and
    the nonce read through this process's mapping, and asserts that each process allocated one
    arena chunk, mapped each peer chunk once, freed nothing, and that every peer's region stays
    at the same mapped address while the nonce seen through it is the current session's."""
    import json

    key = sorted(k for k in MAN["multi"] if MAN["multi"][k]["world"] == 2)[0]
    with tempfile.TemporaryDirectory() as td:
        log = os.path.join(td, "sessions.jsonl")
        torch.multiprocessing.spawn(_worker, args=(2, key, os.path.join(td, "init"), False, 3, 40, log), nprocs=2,
                                    join=True)
        recs = [json.loads(x) for x in open(log)]
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "ipc_sessions.jsonl")
    try:
        os.makedirs(os.path.dirname(out), exist_ok=True)
        with open(out, "w") as f:
            f.writelines(json.dumps(r) + "\n" for r in recs)
    except OSError:
        pass
    assert len(recs) == 3 * 2 * 2
    for rank in (0, 1):
        mine = [r for r in recs if r["rank"] == rank]
        for r in mine:
            assert r["nonce_seen"] == r["announced_nonce"], r
            assert r["arena"][0] == 1 and r["arena"][1] == 1 and r["arena"][3] == 0, r  # no free / re-map
        peer = 1 - rank
        vas = {r["peer_va"] for r in mine if r["peer"] == peer}
        assert len(vas) == 1, mine  # the same mapped region every session
        nonces = [r["announced_nonce"] for r in mine if r["peer"] == peer]
        assert len(set(nonces)) == 3, nonces  # a fresh nonce per session


def _nonce_worker(rank_id, initfile):
    from powersgd_amd import Config, PowerSGD

    torch.distributed.init_process_group("gloo", init_method=f"file://{initfile}", rank=rank_id, world_size=2)
    try:
        dev = torch.device("cuda:0")
        psgd = PowerSGD([torch.zeros(64, 32, device=dev)], Config(2, 1, 2, 0))
        plan = psgd._powersgd._plan
        h = plan.ipc_create(0)
        hs = [None, None]
        torch.distributed.all_gather_object(hs, h)
        peer = 1 - rank_id
        # negative control: the peer's handle announces another session's nonce than the one its
        # buffer holds (what a stale mapping of an earlier buffer looks like): the open refuses
        bad = list(hs)
        nonce = int.from_bytes(bad[peer][-4:], "little")
        bad[peer] = bad[peer][:-4] + (nonce ^ 0x10).to_bytes(4, "little")
        with pytest.raises(RuntimeError, match="stale IPC mapping"):
            plan.ipc_open(2, rank_id, bad)
        # this rank's own entry must be its own handle
        own = list(hs)
        own[rank_id] = own[rank_id][:-4] + (int.from_bytes(own[rank_id][-4:], "little") ^ 0x10).to_bytes(4, "little")
        with pytest.raises(ValueError, match="own exchange handle"):
            plan.ipc_open(2, rank_id, own)
        plan.ipc_open(2, rank_id, hs)  # the true list opens
        torch.distributed.barrier()
        plan.ipc_close()
        torch.distributed.barrier()
    finally:
        torch.distributed.destroy_process_group()


def test_ipc_open_checks_session_nonce():
    with tempfile.TemporaryDirectory() as td:
        torch.multiprocessing.spawn(_nonce_worker, args=(os.path.join(td, "init"),), nprocs=2, join=True)


def _timeout_worker(rank_id, initfile):
    os.environ["PSGD_COMM"] = "ipc"
    os.environ["PSGD_IPC_SPIN"] = "4000"  # ~1 ms of polling
    from powersgd_amd import Config, PowerSGD

    torch.distributed.init_process_group("gloo", init_method=f"file://{initfile}", rank=rank_id, world_size=2)
    try:
        dev = torch.device("cuda:0")
        shapes = [(64, 32), (32, 16)]
        psgd = PowerSGD([torch.zeros(s, device=dev) for s in shapes], Config(2, 1, 2, 0))
        psgd._powersgd._ipc_setup(0)
        if rank_id == 0:  # rank 1 never takes the step: rank 0's waits give up, no hang
            out = psgd.aggregate([torch.randn(s, device=dev) for s in shapes])
            # a second step enqueued before the first one's wait has given up is accepted by the
            # host check; its exchanges see the device copy of the error word and skip the wait
            try:
                out2 = psgd.aggregate([torch.randn(s, device=dev) for s in shapes])
            except RuntimeError as e:  # the first wait had already given up: refused
                assert "timed out" in str(e)
                out2 = None
            torch.cuda.synchronize()
            # invalid sums come back as NaN, never as plausible stale values
            for o in out + (out2 or []):
                assert torch.isnan(o).any(), o
            assert psgd._powersgd.ipc_status()
            assert psgd._powersgd.ipc_status()  # sticky: the exchange stays invalid
            # the next step refuses to run on an invalid exchange instead of returning stale sums
            with pytest.raises(RuntimeError, match="timed out"):
                psgd.aggregate([torch.randn(s, device=dev) for s in shapes])
        psgd._powersgd.close_ipc()
        assert not psgd._powersgd.ipc_status()
    finally:
        torch.distributed.destroy_process_group()


def test_ipc_wait_is_bounded():
    with tempfile.TemporaryDirectory() as td:
        torch.multiprocessing.spawn(_timeout_worker, args=(os.path.join(td, "init"),), nprocs=2, join=True)


def _one_rank_worker(_, initfile, cfg, steps):
    """The IPC exchange path with one rank (own buffer only) against the CPU oracle per step:
    the BASELINE shapes, incl. four power iterations (the rank-1 norm fold of every iteration)."""
    os.environ["PSGD_COMM"] = "ipc"
    from oracle import powersgd_oracle as O
    from powersgd_amd import Config, PowerSGD
    from powersgd_amd.workloads import CONFIGS, hash_tensors

    torch.distributed.init_process_group("gloo", init_method=f"file://{initfile}", rank=0, world_size=1)
    try:
        dev = torch.device("cuda:0")
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
            new = [torch.from_numpy(f) for f in hash_tensors(shapes, seed=700 + t)]
            gd = [(r.float() + x.to(dev)).to(dt) for r, x in zip(res_d, new)]
            # the oracle sees exactly the device inputs (bf16: the rounded values, upcast)
            gc = [g.float().cpu() for g in gd] if dt == torch.bfloat16 else [r + x for r, x in zip(res_c, new)]
            scale = [g.clone() for g in gc]
            od = psgd.aggregate(gd)
            oc = O.policy_step(ora, gc)
            torch.cuda.synchronize()
            for i, g in enumerate(scale):
                tol = (1e-6 if c["rank"] == 1 else 1e-5) if t == 0 else 1e-4
                if dt == torch.bfloat16:
                    tol = 4e-3  # bf16 gradient storage; ~1.1e-3 RMS rounding
                eo = float((od[i].cpu().double() - oc[i].double()).norm()) / max(float(g.norm()), 1e-30)
                er = float((gd[i].cpu().double() - gc[i].double()).norm()) / max(float(g.norm()), 1e-30)
                check(eo, tol, cfg, 0, t, i, "ipc1-out")
                check(er, tol, cfg, 0, t, i, "ipc1-res")
            res_d, res_c = gd, gc
        assert not psgd._powersgd.ipc_status()
        psgd._powersgd.close_ipc()
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.parametrize("cfg", ["cfg2_resnet50_r1", "cfg5_lstm_r1_i4", "cfg3_resnet50_r4", "cfg4_llama_r2_bf16"])
def test_ipc_one_rank_vs_oracle(cfg):
    with tempfile.TemporaryDirectory() as td:
        torch.multiprocessing.spawn(_one_rank_worker, args=(os.path.join(td, "init"), cfg, 3), nprocs=1, join=True)


def _arena_worker(_, initfile):
    """One process (W = 1 over the IPC exchange), several codecs of different sizes: two sessions
    open at once, then a larger one after both closed, then a small one again. Every session is
    checked against the CPU oracle for two steps; the process's exchange arena must serve them from
    regions of its chunks (never freeing one) and re-use the regions the closed sessions returned."""
    os.environ["PSGD_COMM"] = "ipc"
    from oracle import powersgd_oracle as O
    from powersgd_amd import Config, PowerSGD
    from powersgd_amd.workloads import CONFIGS, hash_tensors

    torch.distributed.init_process_group("gloo", init_method=f"file://{initfile}", rank=0, world_size=1)
    try:
        dev = torch.device("cuda:0")

        def make(cfg):
            c = CONFIGS[cfg]
            shapes = c["shapes"]
            psgd = PowerSGD([torch.zeros(s, device=dev) for s in shapes], Config(c["rank"], c["mcr"], c["iters"], 0))
            ora = O.policy_init([torch.zeros(s) for s in shapes], c["rank"], c["mcr"], c["iters"], 0)
            ora.codec.p_flat.copy_(psgd._powersgd._ps_buffer.cpu())
            ora.codec.q_flat.copy_(psgd._powersgd._qs_buffer.cpu())
            return psgd, ora, shapes, c

        def steps(psgd, ora, shapes, c, seed):
            for t in range(2):
                new = [torch.from_numpy(f) for f in hash_tensors(shapes, seed=seed + t)]
                gd = [x.to(dev) for x in new]
                gc = [x.clone() for x in new]
                od = psgd.aggregate(gd)
                oc = O.policy_step(ora, gc)
                torch.cuda.synchronize()
                for i, x in enumerate(new):
                    tol = (1e-6 if c["rank"] == 1 else 1e-5) if t == 0 else 1e-4
                    s = max(float(x.norm()), 1e-30)
                    check(float((od[i].cpu() - oc[i]).norm()) / s, tol, c["rank"], seed, t, i, "arena-out")
                    check(float((gd[i].cpu() - gc[i]).norm()) / s, tol, c["rank"], seed, t, i, "arena-res")

        def info(psgd):
            return psgd._powersgd._plan.ipc_debug(0)

        a = make("cfg5_lstm_r1_i4")
        b = make("cfg2_resnet50_r1")
        steps(*a, seed=900)
        steps(*b, seed=910)  # both sessions open at once: two regions
        ia, ib = info(a[0]), info(b[0])
        assert ia["own_va"] != ib["own_va"] and ia["arena_frees"] == 0
        a[0].close()
        b[0].close()
        va_a = ia["own_va"]
        del a, b
        gc.collect()
        c3 = make("cfg3_resnet50_r4")  # larger factors: a region of its own size
        steps(*c3, seed=920)
        i3 = info(c3[0])
        c3[0].close()
        del c3
        gc.collect()
        a2 = make("cfg5_lstm_r1_i4")  # the small plan again: a region the arena got back
        steps(*a2, seed=930)
        i5 = info(a2[0])
        assert i5["arena_frees"] == 0 and i5["arena_reuses"] >= 2, i5
        assert i5["own_va"] == va_a or i5["own_va"] == i3["own_va"], (i5, va_a, i3)
        a2[0].close()
    finally:
        torch.distributed.destroy_process_group()


def test_ipc_arena_regions_of_different_sizes():
    with tempfile.TemporaryDirectory() as td:
        torch.multiprocessing.spawn(_arena_worker, args=(os.path.join(td, "init"),), nprocs=1, join=True)
