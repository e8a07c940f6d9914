"""bench.py's multi-rank launcher (CPU, gloo): `--gpus N` must start N ranks or fail loudly.

The driver runs `python bench.py --gpus N` (or torch.distributed.run ... bench.py --gpus N);
either way rank 0 must report the process group's real size. `--launch-check` stops after the
rendezvous, so this runs without a GPU."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(PSGD_BENCH_BACKEND="gloo", OMP_NUM_THREADS="1", **kw)
    return env


def test_bench_gpus2_spawns_two_ranks():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # one JSON line, rank 0 only
    assert json.loads(lines[0])["n_gpus"] == 2


def test_bench_rank_count_mismatch_fails():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"],
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 3
    assert "--gpus 2" in p.stderr
