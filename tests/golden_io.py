"""Helpers to read the golden fixtures (tests/golden, written by make_golden.py)."""
from __future__ import annotations

import json
import os
from typing import Dict, List

import numpy as np
import torch

from powersgd_amd.workloads import CONFIGS, hash_normal, hash_tensors

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def manifest() -> dict:
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def load(name: str) -> Dict[str, np.ndarray]:
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def scenario_inputs(meta: dict, step: int, prev_residuals: List[torch.Tensor], rank_id: int = 0,
                    dtype=torch.float32) -> List[torch.Tensor]:
    """Rebuild step ``step``'s input: previous residual + fresh hash gradient (make_golden.py)."""
    shapes = [tuple(s) for s in meta["shapes"]]
    fresh = hash_tensors(shapes, seed=1000 + step + 100 * rank_id)
    zero_at = meta.get("zero_at")
    out = []
    for i, (r, f) in enumerate(zip(prev_residuals, fresh)):
        g = r.clone()
        g.add_(torch.from_numpy(f).to(dtype))
        if zero_at is not None and zero_at[0] == step and i in zero_at[1]:
            g.zero_()
        out.append(g)
    return out


def config_state0(p_numel: int, q_numel: int):
    return (torch.from_numpy(hash_normal(7, p_numel, stream=1)),
            torch.from_numpy(hash_normal(7, q_numel, stream=2)))


def config_grads(cfg: str, step: int, prev: List[torch.Tensor]) -> List[torch.Tensor]:
    c = CONFIGS[cfg]
    fresh = hash_tensors(c["shapes"], seed=2000 + step)
    out = []
    for g, f in zip(prev, fresh):
        ft = torch.from_numpy(f)
        if c["dtype"] == "bf16":
            ft = ft.to(torch.bfloat16).float()
        g = g.clone() + ft
        if c["dtype"] == "bf16":
            g = g.to(torch.bfloat16).float()
        out.append(g)
    return out


def checksums(arr: np.ndarray, nsamp: int = 256):
    a = arr.astype(np.float64).reshape(-1)
    idx = np.linspace(0, a.size - 1, num=min(nsamp, a.size)).astype(np.int64)
    return a.sum(), np.sqrt((a * a).sum()), a[idx]
