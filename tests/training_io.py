"""Helpers for the training-loop fixtures (tests/golden/make_golden_training.py)."""
from __future__ import annotations

import json
import os

import torch

from golden_io import GOLDEN, load  # noqa: F401
from powersgd_amd.workloads import hash_tensors


def training_manifest() -> dict:
    with open(os.path.join(GOLDEN, "training_manifest.json")) as f:
        return json.load(f)


TMAN = training_manifest()
SHAPES = [tuple(s) for s in TMAN["shapes"]]


def init_params():
    """make_golden_training.init_params."""
    return [torch.from_numpy(x.copy()) * TMAN["param_scale"] for x in hash_tensors(SHAPES, seed=TMAN["param_seed"])]


def step_grads(t: int, rank_id: int):
    """make_golden_training.step_grads: rank `rank_id`'s fresh gradient of step t."""
    return [torch.from_numpy(x) for x in hash_tensors(SHAPES, seed=TMAN["grad_seed"] + 10 * t + rank_id)]
