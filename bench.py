"""Benchmark of the PowerSGD hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config NAME] [--sets S]

One step = one ``PowerSGD.aggregate`` over the synthetic gradients of the workload
(compressed matrices: power iterations + factor all-reduce + fused residual/output
pass; uncompressed tensors: flat pack + all-reduce), inputs resident in HBM.

N > 1: one process per GPU. Launched by the driver through ``torch.distributed.run`` (RANK /
WORLD_SIZE / LOCAL_RANK in the environment), or, when started as ``python bench.py --gpus N``
without them, this script starts ``torch.distributed.run`` itself as a child process BEFORE
touching the GPU and exits with its code. Every rank holds its own gradients (data parallel,
weak scaling) and the P/Q factors are SUM-all-reduced over RCCL. A rank count that differs from
``--gpus`` is an error (exit 3).

Cache state. The headline is COLD: the timed loop rotates over S (default 4) independent
gradient sets, so between two uses of one set the other S-1 sets (gradients read and rewritten,
fresh outputs written) stream > 256 MiB through the chip and the set is out of the 256 MiB
Infinity Cache, as after a real backward pass. The same loop on ONE set (warm: the 102 MB
ResNet-50 set plus its output fit the Infinity Cache) is reported beside it.

Prints ONE JSON line on rank 0. ``value`` = gradient bytes processed by all ranks per second
(GB/s, cold). ``roofline`` = the final pass, the dominant kernel: k_final_odd (the last odd
power iteration fused with the residual/output writes) or k_apply, timed with HIP events that
the library records on the launch stream around every such launch, over a second pass of the
same cold rotation. ``cpu_baseline`` = the CPU oracle (bit-identical restatement of the
reference) on a bounded sample, rank 0 at N = 1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)


def parse():
    from powersgd_amd.workloads import CONFIGS

    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="cfg2_resnet50_r1", choices=sorted(CONFIGS))
    ap.add_argument("--sets", type=int, default=4, help="gradient sets rotated in the cold loop")
    ap.add_argument("--iters", type=int, default=None,
                    help="experiments only: override the config's num_iters_per_step (reported in config)")
    ap.add_argument("--mode", default="both", choices=["both", "cold", "warm"],
                    help="profiling runs: time only one cache state (the headline needs 'both' or 'cold')")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the rank4/cfg4/cfg5 blocks and (N = 1) the world-size > 1 path block")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-parity", action="store_true",
                    help="N > 1: skip the cross-GPU parity check of the W > 1 transports (after the timed blocks)")
    ap.add_argument("--launch-check", action="store_true",
                    help="rendezvous + world-size report only (no codec; CPU-testable with gloo)")
    return ap.parse_args()


def numel(s):
    n = 1
    for d in s:
        n *= d
    return n


def apply_alg_bytes(c, mask, world, fused):
    """Algorithmic HBM bytes of ONE final-pass launch + the factor panels it must read (fp32).
    k_apply: read G0, write residual, write output (s bytes each per element).
    k_final_odd (fused last odd iteration): read G0, write residual, and at world size 1
    write the output (2 or 3 s bytes per element). At world size 1 the same launch also
    packs the uncompressed tensors (read, write flat, write zero: 3 s bytes per element)."""
    s = 2 if c["dtype"] == "bf16" else 4
    terms = 1 if world == 1 else 2
    per = 3 if (not fused or world == 1) else 2
    total = 0
    for shp, comp in zip(c["shapes"], mask):
        if not comp:
            if world == 1:
                total += 3 * s * numel(shp)
            continue
        n = shp[0]
        m = numel(shp) // n
        r = min(c["rank"], n, m)
        total += per * s * n * m + 4 * terms * c["iters"] * r * (n + m)
    return total


def step_alg_bytes(c, mask, world, fused):
    """sum_c s*n*m*(I+3) + sum_c 4*I*r*(n+m) + sum_u 3*s*N. With the fused
    last odd iteration the gradient is read once less: (I+2) instead of (I+3)."""
    s = 2 if c["dtype"] == "bf16" else 4
    passes = c["iters"] + (2 if fused else 3)
    total = 0
    for shp, comp in zip(c["shapes"], mask):
        N = numel(shp)
        if comp:
            n = shp[0]
            m = N // n
            r = min(c["rank"], n, m)
            total += s * N * passes + 4 * c["iters"] * r * (n + m)
        else:
            total += 3 * s * N
    return total


def load_pmc_traffic(cfg, cache):
    """HBM traffic per final-pass launch from the committed rocprofv3 --pmc passes."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    return d.get(f"{cfg}:{cache}", d.get(cfg) if cache == "warm" else None)


def cpu_baseline(c, seconds):
    from oracle import powersgd_oracle as O

    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    cores = max(1, min(int(os.environ.get("OMP_NUM_THREADS", cores)), cores))
    torch.set_num_threads(cores)
    g = torch.Generator().manual_seed(0)
    shapes = c["shapes"]
    grads = [torch.randn(s, generator=g) for s in shapes]
    ps = O.policy_init([torch.zeros(s) for s in shapes], c["rank"], c["mcr"], c["iters"], 0)
    O.policy_step(ps, grads)  # warm-up
    times = []
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end or len(times) < 3:
        t0 = time.perf_counter()
        O.policy_step(ps, grads)
        times.append(time.perf_counter() - t0)
    s = 2 if c["dtype"] == "bf16" else 4
    byts = sum(numel(x) for x in shapes) * s
    t = statistics.median(times)
    return {"value": round(byts / t / 1e9, 4), "unit": "GB/s", "cores": cores, "kind": "port",
            "sample": f"{len(times)} oracle aggregate() steps of {c['name']} (fp32 CPU, median step "
                      f"{t*1e3:.1f} ms, {sum(times):.1f} s total)"}


def launch_ranks(a) -> int:
    """Start one rank per GPU with torch.distributed.run as a CHILD process (this process has
    not touched the GPU: no exec from a GPU-initialised process) and return its exit code."""
    import socket

    with socket.socket() as sk:  # a free rendezvous port on the loopback interface
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def timed(fn, steps, world, dev):
    """Barrier + synchronize on both sides of `steps` calls; max wall time over ranks."""
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        fn(k)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def main():
    a = parse()
    # bounded device-side waits of the IPC exchange blocks: ~1 s per wait (default ~18 s)
    os.environ.setdefault("PSGD_IPC_SPIN", str(1 << 22))
    env_world = os.environ.get("WORLD_SIZE")
    if a.gpus > 1 and env_world is None:
        sys.exit(launch_ranks(a))
    # stdout carries exactly ONE JSON line: anything else printed at the C level (RCCL's
    # version banner at communicator init) goes to stderr
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but the launcher started {world} rank(s)", file=sys.stderr)
        sys.exit(3)
    backend = os.environ.get("PSGD_BENCH_BACKEND", "nccl")
    if a.launch_check:  # launcher + rendezvous only (CPU test with PSGD_BENCH_BACKEND=gloo)
        if world > 1:
            torch.distributed.init_process_group(backend)
            world = torch.distributed.get_world_size()
        if rank == 0:
            os.write(json_fd, (json.dumps({"n_gpus": world, "backend": backend if world > 1 else None}) + "\n").encode())
        if world > 1:
            torch.distributed.destroy_process_group()
        return

    if world > 1:
        # rehearsal knobs for a one-GPU box (never set by the driver): every rank on cuda:0
        # over gloo exercises the N > 1 code path end to end; the real run is RCCL, one GPU
        # per rank
        if os.environ.get("PSGD_BENCH_ONE_DEVICE") == "1":
            local = 0
        torch.cuda.set_device(local)
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.distributed.init_process_group(backend)
        got = torch.distributed.get_world_size()
        if got != a.gpus:
            print(f"bench.py: process group reports {got} ranks, --gpus {a.gpus}", file=sys.stderr)
            sys.exit(3)
    dev = torch.device("cuda", local)
    out = measure(a, a.config, world, rank, dev, backend, a.mode)
    if world > 1 and os.environ.get("PSGD_BENCH_IPC", "1") == "1" and "PSGD_COMM" not in os.environ:
        # the same step with every factor all-reduce as a one-shot sum over IPC exchange buffers
        # (device-side flags, no collective library): beside the RCCL headline, not instead of it
        out["ipc_exchange"] = ipc_block(a, world, rank, dev, backend)
    if rank == 0 and world == 1:
        # the real caller's cache state: autograd's accumulation into p.grad just before
        out["post_backward"] = post_backward(a, a.config, dev)
    if not a.no_extra:
        # every other config BASELINE names for this run, at this world size (cold, same steps):
        # rank4 = cfg3, the north-star ResNet-50 rank-4 config ("rank=1/4 ... at 1 and 8 GPUs");
        # cfg4 = the bf16 Llama linears; cfg5 = the LSTM matrix at four power iterations (four
        # collectives per step at N > 1). All ranks take part (collective timing at N > 1).
        for key, cfg in EXTRA_BLOCKS:
            if cfg == a.config:
                continue
            m = measure(a, cfg, world, rank, dev, backend, "cold")
            # every block carries its final pass's kernel roofline (events on the codec's stream,
            # PMC traffic from profiles/pmc_traffic.json where measured) beside the step's
            keep = ("value", "ms_per_step", "per_rank_GBs", "roofline", "step_roofline")
            out[key] = {k: m[k] for k in keep}
            out[key]["config"] = m["config"]
            if rank == 0 and world == 1 and key == "rank4":
                out[key]["post_backward"] = post_backward(a, cfg, dev)
    if world > 1 and not a.no_parity:
        # correctness of the cross-device run itself (after every timed block)
        out["multi_gpu_parity"] = multi_gpu_parity(world, rank, dev, backend)
    if rank == 0 and world == 1 and not a.no_extra:
        # the world-size > 1 code path (bucketed async factor all-reduces, per-bucket kernels,
        # write-only output pass) timed on this one GPU through a 1-rank RCCL group: the
        # per-rank compute floor of every multi-GPU point (no xGMI traffic: one rank)
        out["w_gt1_path"] = one_rank_group(a, dev)
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        c = dict(CONFIGS_()[a.config])
        c["name"] = a.config
        if a.iters is not None:
            c["iters"] = a.iters
        out["cpu_baseline"] = cpu_baseline(c, a.cpu_seconds)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if world > 1:
        torch.distributed.destroy_process_group()


EXTRA_BLOCKS = (("rank4", "cfg3_resnet50_r4"), ("cfg4", "cfg4_llama_r2_bf16"), ("cfg5", "cfg5_lstm_r1_i4"))


def CONFIGS_():
    from powersgd_amd.workloads import CONFIGS

    return CONFIGS


# ------------------------------------------------------------------ multi-GPU parity (N > 1)
# The driver's N > 1 run is the only cross-device execution of the W > 1 transports, so after
# every timed block (never inside one) each transport runs PARITY_STEPS steps of the ResNet-50
# configs from one common injected P/Q state; every rank's outputs and residuals are gathered to
# rank 0 and compared with W reference workers (oracle/multiworker.py: the CPU restatement of the
# reference, W threads meeting at the reference's SUM all-reduce, powersgd.py:204-219). The
# oracle is the checker here, never the thing measured.
PARITY_STEPS = 2
# every config BASELINE names for the multi-GPU runs (cfg3: rank 4; cfg4: bf16 with 11008-column
# rows; cfg5: four power iterations, i.e. four collectives per step) and the headline cfg2
PARITY_CFGS = tuple(os.environ.get("PSGD_PARITY_CFGS", "cfg2_resnet50_r1,cfg3_resnet50_r4,cfg4_llama_r2_bf16,"
                                                       "cfg5_lstm_r1_i4").split(","))
PARITY_TOL = (1e-5, 1e-4)  # fp32: step 0 (same state), step 1 (free-running)
PARITY_TOL_BF16 = (4e-3, 4e-3)  # bf16 gradient storage (the residual is stored in bf16)


def parity_inputs(shapes, rank, t):
    """Rank `rank`'s fresh gradient of step t (CPU fp32, seeded: rank 0 regenerates every rank's)."""
    g = torch.Generator().manual_seed(7919 * (rank + 1) + 104729 * (t + 1))
    return [torch.randn(s, generator=g) for s in shapes]


def gather_to_rank0(t, world, rank, backend):
    """Every rank's 1-D tensor, in rank order, on rank 0 (CPU); None on the other ranks."""
    if backend == "nccl":
        parts = [torch.empty_like(t) for _ in range(world)]
        torch.distributed.all_gather(parts, t)
        return [p.cpu() for p in parts] if rank == 0 else None
    t = t.detach().cpu()
    parts = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
    torch.distributed.gather(t, parts, dst=0)
    return parts


def parity_collect(step, shapes, world, rank, backend, dev, dtype=torch.float32):
    """PARITY_STEPS steps of `step(grads) -> outs` on this rank (error feedback: the residual
    left in `grads` + the next fresh gradient, added in fp32 and stored in `dtype`), then the
    gathers. Every rank makes the same collectives even if its steps failed (its rows are NaN
    then), so a failure cannot hang the others. Returns (outs[t][w], residuals[t][w], errors[w])
    on rank 0."""
    total = sum(numel(s) for s in shapes)
    flats, err = [], None
    try:
        res = [torch.zeros(s, device=dev, dtype=dtype) for s in shapes]
        for t in range(PARITY_STEPS):
            g = [(r.float() + x.to(dev)).to(dtype) for r, x in zip(res, parity_inputs(shapes, rank, t))]
            o = step(g)
            flats.append((torch.cat([x.reshape(-1).float() for x in o]), torch.cat([x.reshape(-1).float() for x in g])))
            res = g
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
    except Exception as e:  # reported, not raised: the other ranks still gather
        err = f"{type(e).__name__}: {str(e)[:300]}"
        flats = [(torch.full((total,), float("nan"), device=dev),) * 2 for _ in range(PARITY_STEPS)]
    errs = [None] * world
    torch.distributed.all_gather_object(errs, err)
    outs = [gather_to_rank0(o, world, rank, backend) for o, _ in flats]
    ress = [gather_to_rank0(r, world, rank, backend) for _, r in flats]
    return outs, ress, errs


def _nanmax(a, b):
    return b if (b != b or b > a) else a


def parity_check(c, world, p0, q0, outs, ress):
    """Rank 0: the reference's W-worker steps on the same inputs from the same P/Q state; the
    largest per-tensor error relative to that rank's input tensor (SURVEY §8(c) metric). bf16
    configs: each worker's input is exactly the device's (its gathered bf16 residual + the fresh
    gradient, rounded to bf16), upcast to fp32 for the oracle (the reference raises on bf16)."""
    from oracle import multiworker as MW
    from oracle import powersgd_oracle as O

    shapes = c["shapes"]
    sizes = [numel(s) for s in shapes]
    bf16 = c.get("dtype") == "bf16"
    tols = PARITY_TOL_BF16 if bf16 else PARITY_TOL
    states = []
    for _ in range(world):
        st = O.policy_init([torch.zeros(s) for s in shapes], c["rank"], c["mcr"], c["iters"], 0)
        st.codec.p_flat.copy_(p0)
        st.codec.q_flat.copy_(q0)
        states.append(st)
    res = [[torch.zeros(s) for s in shapes] for _ in range(world)]
    steps, ok, same = [], True, True
    for t in range(PARITY_STEPS):
        if bf16:
            prev = [[torch.zeros(s) for s in shapes] if t == 0 else
                    [x.view(s) for x, s in zip(torch.split(ress[t - 1][w], sizes), shapes)] for w in range(world)]
            grads = [[(r + x).bfloat16().float() for r, x in zip(prev[w], parity_inputs(shapes, w, t))]
                     for w in range(world)]
        else:
            grads = [[r + x for r, x in zip(res[w], parity_inputs(shapes, w, t))] for w in range(world)]
        scale = [[max(float(g.norm()), 1e-30) for g in gw] for gw in grads]
        want = MW.run_workers(states, grads)
        eo = er = 0.0
        for w in range(world):
            got_o = torch.split(outs[t][w], sizes)
            got_r = torch.split(ress[t][w], sizes)
            for i in range(len(shapes)):
                # NaN-propagating maximum (max() would keep the earlier value)
                eo = _nanmax(eo, float((got_o[i] - want[w][i].reshape(-1)).norm()) / scale[w][i])
                er = _nanmax(er, float((got_r[i] - grads[w][i].reshape(-1)).norm()) / scale[w][i])
            same = same and torch.equal(outs[t][w], outs[t][0])
        tol = tols[min(t, 1)]
        ok = ok and eo <= tol and er <= tol  # NaN compares False
        steps.append({"max_rel_out": float(f"{eo:.3e}"), "max_rel_res": float(f"{er:.3e}"), "tol": tol})
        res = grads
    return {"ok": ok, "outputs_equal_on_all_ranks": same, "steps": steps}


def multi_gpu_parity(world, rank, dev, backend):
    """Each W > 1 transport (RCCL in the library and the IPC exchange on the nccl backend;
    torch.distributed and the IPC exchange on gloo) on the ResNet-50 configs, checked on rank 0."""
    from powersgd_amd import Config, PowerSGD

    transports = ("rccl", "ipc") if backend == "nccl" else ("torch", "ipc")
    if os.environ.get("PSGD_PARITY_TRANSPORTS"):  # diagnostics: a subset
        transports = tuple(t for t in transports if t in os.environ["PSGD_PARITY_TRANSPORTS"].split(","))
    report = {"steps": PARITY_STEPS, "world": world,
              "note": "every rank's outputs/residuals vs W reference workers from one injected P/Q state"}
    for tr in transports:
        old = os.environ.get("PSGD_COMM")
        os.environ["PSGD_COMM"] = tr
        report[tr] = {}
        try:
            for cfg in PARITY_CFGS:
                c = CONFIGS_()[cfg]
                dtype = torch.bfloat16 if c["dtype"] == "bf16" else torch.float32
                psgd = PowerSGD([torch.zeros(s, device=dev, dtype=dtype) for s in c["shapes"]],
                                Config(c["rank"], c["mcr"], c["iters"], 0))
                codec = psgd._powersgd
                for buf in (codec._ps_buffer, codec._qs_buffer):  # one common injected state
                    host = buf.cpu()
                    torch.distributed.broadcast(host if backend != "nccl" else buf, src=0)
                    if backend != "nccl":
                        buf.copy_(host)
                p0, q0 = codec._ps_buffer.cpu(), codec._qs_buffer.cpu()
                outs, ress, errs = parity_collect(psgd.aggregate, c["shapes"], world, rank, backend, dev, dtype)
                # an IPC wait that gave up invalidates the sums (NaN): report it before close()
                # clears the sticky status
                waits = [None] * world
                torch.distributed.all_gather_object(waits, bool(codec._ipc_open and codec.ipc_status()))
                if any(waits):
                    errs = errs + [f"IPC exchange wait timed out on rank(s) {[r for r, w in enumerate(waits) if w]}"]
                try:
                    codec.close()
                except RuntimeError as e:
                    errs = errs + [str(e)[:200]]
                if rank == 0:
                    r = parity_check(c, world, p0, q0, outs, ress)
                    if any(errs):
                        r["ok"] = False
                        r["errors"] = [e for e in errs if e]
                    report[tr][cfg] = r
                del psgd, codec
                torch.cuda.empty_cache()
        finally:
            if old is None:
                os.environ.pop("PSGD_COMM", None)
            else:
                os.environ["PSGD_COMM"] = old
    if rank == 0:
        report["ok"] = all(report[tr][cfg]["ok"] for tr in transports for cfg in PARITY_CFGS)
    return report


def post_backward(a, cfg_name, dev):
    """The real caller's cache state (reference README.md:39-42: ``loss.backward()`` accumulates
    the fresh gradient into ``p.grad``, which holds the residual, right before ``aggregate``).
    Per step an in-stream foreach add of a fresh gradient set into the gradients, then one
    aggregate; CUDA events on torch's current stream (the codec's launch stream) bracket the
    aggregate alone, so the add is not counted but its cache footprint is."""
    from powersgd_amd import Config, PowerSGD

    c = dict(CONFIGS_()[cfg_name])
    dtype = torch.bfloat16 if c["dtype"] == "bf16" else torch.float32
    shapes = c["shapes"]
    gen = torch.Generator(device=dev).manual_seed(4321)
    grads = [torch.randn(s, generator=gen, device=dev, dtype=torch.float32).to(dtype) for s in shapes]
    fresh = [torch.randn(s, generator=gen, device=dev, dtype=torch.float32).to(dtype) for s in shapes]
    psgd = PowerSGD([torch.zeros(s, device=dev, dtype=dtype) for s in shapes], Config(c["rank"], c["mcr"], c["iters"], 0))
    for _ in range(a.warmup):
        torch._foreach_add_(grads, fresh)
        psgd.aggregate(grads)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    torch.cuda.synchronize()
    for k in range(a.steps):
        torch._foreach_add_(grads, fresh)  # autograd's accumulation into p.grad (the residual)
        evs[k][0].record()
        psgd.aggregate(grads)
        evs[k][1].record()
    torch.cuda.synchronize()
    ms = sum(e0.elapsed_time(e1) for e0, e1 in evs) / a.steps
    s = 2 if dtype == torch.bfloat16 else 4
    byts = sum(numel(x) for x in shapes) * s
    del grads, fresh, psgd
    torch.cuda.empty_cache()
    return {"ms_per_step": round(ms, 4), "value": round(byts / (ms * 1e-3) / 1e9, 3), "unit": "GB/s",
            "note": "in-stream grad += fresh (autograd accumulation) before each aggregate; events around "
                    "aggregate only"}


def ipc_block(a, world, rank, dev, backend):
    os.environ["PSGD_COMM"] = "ipc"
    try:
        m = measure(a, a.config, world, rank, dev, backend, "cold", dist_path=True)
        blk = {k: m[k] for k in ("value", "ms_per_step", "roofline", "step_roofline")}
        blk["timed_out"] = m.get("ipc_timed_out")
        return blk
    except RuntimeError as e:  # setup failures are collective (BasicPowerSGD._ipc_setup)
        return {"error": str(e)[:300]}
    finally:
        del os.environ["PSGD_COMM"]


def env_block(a, world, rank, dev, backend, env):
    """The headline workload again under extra environment knobs (read at plan creation)."""
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        m = measure(a, a.config, world, rank, dev, backend, "cold", dist_path=True)
        blk = {k: m[k] for k in ("value", "ms_per_step", "step_roofline")}
        blk["env"] = env
        blk["buckets"] = m["config"]["buckets"]
        return blk
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def one_rank_group(a, dev):
    """cfg3 and cfg2 through PowerSGD.aggregate with torch.distributed initialised as ONE RCCL
    rank on this GPU: is_distributed() is True, so the exact multi-GPU code path runs."""
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    torch.distributed.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                         device_id=dev)
    try:
        res = {"note": "world-size>1 code path on one GPU via a 1-rank RCCL process group (per-rank compute floor; "
                       "no xGMI traffic)"}
        for cfg in ("cfg3_resnet50_r4", "cfg2_resnet50_r1", "cfg5_lstm_r1_i4"):
            m = measure(a, cfg, 1, 0, dev, "nccl", "cold", dist_path=True)
            res[cfg] = {k: m[k] for k in ("value", "ms_per_step", "roofline", "step_roofline")}
            res[cfg]["buckets"] = m["config"]["buckets"]
        # the IPC exchange path (psgd_aggregate_ipc) of the same configs: its flag handshake and
        # rank-order sums with W = 1 (own buffer only)
        os.environ["PSGD_COMM"] = "ipc"
        try:
            res["ipc_exchange"] = {}
            for cfg in ("cfg3_resnet50_r4", "cfg2_resnet50_r1"):
                m = measure(a, cfg, 1, 0, dev, "nccl", "cold", dist_path=True)
                res["ipc_exchange"][cfg] = {"ms_per_step": m["ms_per_step"], "value": m["value"],
                                            "timed_out": m.get("ipc_timed_out")}
        finally:
            del os.environ["PSGD_COMM"]
        return res
    finally:
        torch.distributed.destroy_process_group()


def measure(a, cfg_name, world, rank, dev, backend, mode, dist_path=False):
    """One workload: warm-up, the timed cold (rotating sets) and warm loops, the final-pass
    roofline pass. `world` is the job's world size (1 for the 1-rank group)."""
    from powersgd_amd import Config, PowerSGD

    CONFIGS = CONFIGS_()
    c = dict(CONFIGS[cfg_name])
    c["name"] = cfg_name
    if a.iters is not None and cfg_name == a.config:
        c["iters"] = a.iters
    dtype = torch.bfloat16 if c["dtype"] == "bf16" else torch.float32
    shapes = c["shapes"]
    S = max(1, a.sets)
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    sets = [[torch.randn(s, generator=gen, device=dev, dtype=torch.float32).to(dtype) for s in shapes]
            for _ in range(S)]
    params = [torch.zeros(s, device=dev, dtype=dtype) for s in shapes]
    psgd = PowerSGD(params, Config(c["rank"], c["mcr"], c["iters"], 0))
    codec = psgd._powersgd

    for k in range(a.warmup):
        psgd.aggregate(sets[k % S])
    torch.cuda.synchronize()
    if codec._ipc_open:
        # the IPC exchange's device-side waits are bounded (PSGD_IPC_SPIN, ~1 s here): if any
        # rank's warm-up wait gave up, every rank abandons the block instead of timing garbage
        bad = [None] * world
        mine = codec.ipc_status()
        if world > 1:
            torch.distributed.all_gather_object(bad, mine)
        else:
            bad = [mine]
        if any(bad):
            codec.close_ipc()
            raise RuntimeError(f"IPC exchange wait timed out during warm-up on rank(s) "
                               f"{[r for r, b in enumerate(bad) if b]}")

    # timed regions: K plain steps each (no instrumentation inside); cold = rotating sets
    do_cold, do_warm = mode in ("both", "cold"), mode in ("both", "warm")
    cold = timed(lambda k: psgd.aggregate(sets[k % S]), a.steps, world, dev) if do_cold else None
    warm = timed(lambda k: psgd.aggregate(sets[0]), a.steps, world, dev) if do_warm else None

    # roofline passes: the same K steps again with HIP events around every final-pass launch,
    # recorded by the library on the launch stream
    def kernel_pass(pick):
        codec._plan.set_timing(True)
        first = codec.step_counter
        for k in range(a.steps):
            psgd.aggregate(sets[pick(k)])
        torch.cuda.synchronize()
        total_ms, launches = codec._plan.timing_read()
        codec._plan.set_timing(False)
        # per STEP: at world size > 1 the final pass is one launch per collective bucket, and
        # the algorithmic bytes below are the whole step's final pass
        return total_ms / a.steps, first, launches / a.steps

    apply_ms_cold, first_cold, lps_cold = kernel_pass(lambda k: k % S) if do_cold else (None, None, None)
    apply_ms_warm, first_warm, lps_warm = kernel_pass(lambda k: 0) if do_warm else (None, None, None)
    if first_cold is None:
        first_cold = first_warm

    multi = world > 1 or dist_path
    s = 2 if dtype == torch.bfloat16 else 4
    grad_bytes = sum(numel(x) for x in shapes) * s
    mask = psgd.is_compressed_mask
    # which final pass each timed step took (I odd: steps alternate between the fused last odd
    # iteration and k_apply); bytes are averaged over the timed steps
    forms = [codec._plan.fused_final(t, not multi) for t in range(first_cold, first_cold + a.steps)]
    nf = sum(1 for f in forms if f)
    frac_f = nf / a.steps
    wb = 2 if multi else 1  # the byte model of the multi-GPU path (no output in the fused pass)
    ab = frac_f * apply_alg_bytes(c, mask, wb, True) + (1 - frac_f) * apply_alg_bytes(c, mask, wb, False)
    sb = frac_f * step_alg_bytes(c, mask, wb, True) + (1 - frac_f) * step_alg_bytes(c, mask, wb, False)
    kf = ("k_final_proj (fused last odd iteration, projection form: G X, residual G - G X X^T, output G X X^T)"
          if nf and all(f == 2 for f in forms if f) else
          "k_final_odd (fused last odd iteration: product + residual" + (")" if multi else " + output)"))
    kname = kf if nf == a.steps else "k_apply (fused residual + output)" if nf == 0 else f"{kf} / k_apply, alternating"

    def roof(apply_ms, cache, lps):
        ach = ab / (apply_ms * 1e-3) / 1e9
        return {"kernel": kname, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4),
                "traffic": load_pmc_traffic(cfg_name, cache) if not multi else None,
                "alg_bytes_per_launch": round(ab), "avg_launch_us": round(apply_ms * 1e3, 2),
                "launches_per_step": round(lps, 2), "cache": cache}

    def step_roof(elapsed):
        ms = elapsed / a.steps * 1e3
        return {"alg_bytes_per_step": round(sb), "achieved_GBs": round(sb / (ms * 1e-3) / 1e9, 1),
                "frac": round(sb / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}

    head = cold if do_cold else warm
    value = world * grad_bytes * a.steps / head / 1e9
    out = {
        "metric": "gradient GB/s compressed+decompressed (device-resident)",
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(head / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
        "data": "synthetic N(0,1) gradients of the named parameter shapes (torch.randn on device), " +
                (f"{S} independent sets rotated per step (cold Infinity Cache)" if do_cold else "one set (warm)"),
        "config": {"workload": cfg_name, "rank": c["rank"], "num_iters_per_step": c["iters"],
                   "min_compression_rate": c["mcr"], "tensors": len(shapes),
                   "compressed_tensors": sum(mask), "gradient_bytes_per_rank": grad_bytes,
                   "parallelism": f"dp{world}", "cache": "cold" if do_cold else "warm",
                   "gradient_sets": S if do_cold else 1,
                   "buckets": len(codec._buckets) if codec._buckets else 1,
                   "backend": (backend if multi else None)},
        "per_rank_GBs": round(value / world, 3),
        "roofline": roof(apply_ms_cold, "cold", lps_cold) if do_cold else roof(apply_ms_warm, "warm", lps_warm),
        "step_roofline": step_roof(head),
    }
    if codec._ipc_open:
        out["ipc_timed_out"] = codec.ipc_status()
        codec.close_ipc()
    if do_cold and do_warm:
        out["warm"] = {"value": round(world * grad_bytes * a.steps / warm / 1e9, 3),
                       "ms_per_step": round(warm / a.steps * 1e3, 4),
                       "roofline": roof(apply_ms_warm, "warm", lps_warm), "step_roofline": step_roof(warm)}
    del sets, params, psgd
    torch.cuda.empty_cache()
    return out


if __name__ == "__main__":
    main()
