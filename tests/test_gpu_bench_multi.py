"""bench.py's N > 1 path end to end on the one-GPU box: two ranks on cuda:0 over gloo
(PSGD_BENCH_ONE_DEVICE=1, the rehearsal knob; the driver's real run is RCCL, one GPU per rank).
The JSON line must carry the cross-rank parity check of every W > 1 transport on that backend
(torch.distributed and the IPC exchange) and report it green."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_one_device_parity():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "PSGD_COMM")}
    env.update(PSGD_BENCH_ONE_DEVICE="1", PSGD_BENCH_BACKEND="gloo", OMP_NUM_THREADS="4")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--sets", "2", "--no-cpu-baseline"], env=env, capture_output=True, text=True, timeout=420)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    rep = json.loads(lines[0])["multi_gpu_parity"]
    print(json.dumps(rep))
    assert rep["world"] == 2 and set(rep) >= {"torch", "ipc"}
    for tr in ("torch", "ipc"):
        for cfg, r in rep[tr].items():
            assert r["ok"], (tr, cfg, r)
            assert r["outputs_equal_on_all_ranks"], (tr, cfg)
    assert rep["ok"]
