"""bench.py's N > 1 path end to end on the one-GPU box: two ranks on cuda:0 over gloo
(PSGD_BENCH_ONE_DEVICE=1, the rehearsal knob; the driver's real run is RCCL, one GPU per rank).
The JSON line must carry the timed blocks of every config BASELINE names for the multi-GPU runs
(rank4 = cfg3, cfg4, cfg5) and the cross-rank parity check of every W > 1 transport on that
backend (torch.distributed and the IPC exchange) on all four configs, green."""
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
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["workload"] == "cfg2_resnet50_r1"
    for key, cfg in (("rank4", "cfg3_resnet50_r4"), ("cfg4", "cfg4_llama_r2_bf16"), ("cfg5", "cfg5_lstm_r1_i4")):
        blk = line[key]
        assert blk["config"]["workload"] == cfg and blk["config"]["parallelism"] == "dp2", (key, blk)
        assert blk["value"] > 0 and blk["ms_per_step"] > 0 and "step_roofline" in blk, (key, blk)
    assert "roofline" in line["rank4"]
    rep = line["multi_gpu_parity"]
    print(json.dumps(rep))
    assert rep["world"] == 2 and set(rep) >= {"torch", "ipc"}
    want = {"cfg2_resnet50_r1", "cfg3_resnet50_r4", "cfg4_llama_r2_bf16", "cfg5_lstm_r1_i4"}
    for tr in ("torch", "ipc"):
        assert set(rep[tr]) == want, (tr, sorted(rep[tr]))
        for cfg, r in rep[tr].items():
            assert r["ok"], (tr, cfg, r)
            assert r["outputs_equal_on_all_ranks"], (tr, cfg)
    assert rep["ok"]
