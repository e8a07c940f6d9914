"""Synthetic gradient workloads named in BASELINE.json, and a portable input generator.

The shapes are the parameter shapes of the models the reference is benchmarked
on (README.md:26 uses torchvision ResNet-50). torchvision is not installed, so
the ResNet-50 parameter list is written out here in ``model.parameters()`` order.

``hash_normal`` is a counter-based N(0,1) generator (splitmix64 + Box-Muller in
numpy). It does not depend on torch RNG internals, so the same inputs can be
regenerated on any machine for parity checks against committed checksums.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np

Shape = Tuple[int, ...]


def resnet50_shapes(num_classes: int = 1000) -> List[Shape]:
    """torchvision resnet50 parameter shapes, in ``model.parameters()`` order (161 tensors)."""
    out: List[Shape] = [(64, 3, 7, 7), (64,), (64,)]
    inplanes = 64
    for planes, blocks in ((64, 3), (128, 4), (256, 6), (512, 3)):
        for b in range(blocks):
            out += [(planes, inplanes, 1, 1), (planes,), (planes,)]
            out += [(planes, planes, 3, 3), (planes,), (planes,)]
            out += [(planes * 4, planes, 1, 1), (planes * 4,), (planes * 4,)]
            if b == 0:
                out += [(planes * 4, inplanes, 1, 1), (planes * 4,), (planes * 4,)]
            inplanes = planes * 4
    out += [(num_classes, 2048), (num_classes,)]
    return out


def reference_test_model_shapes() -> List[Shape]:
    """The model of the reference's own unit tests (tests/powersgd_test.py:5-11)."""
    return [(100, 3, 3, 3), (100,), (50, 100, 5, 5), (50,), (1, 50), (1,)]


# BASELINE.json "configs" (index = position in that list).
CONFIGS: Dict[str, dict] = {
    "cfg1_1024sq_r1": dict(shapes=[(1024, 1024)], rank=1, iters=2, mcr=2, dtype="f32"),
    "cfg2_resnet50_r1": dict(shapes=resnet50_shapes(), rank=1, iters=2, mcr=2, dtype="f32"),
    "cfg3_resnet50_r4": dict(shapes=resnet50_shapes(), rank=4, iters=2, mcr=2, dtype="f32"),
    "cfg4_llama_r2_bf16": dict(
        shapes=[(4096, 4096), (4096, 11008)], rank=2, iters=1, mcr=10, dtype="bf16"
    ),
    "cfg5_lstm_r1_i4": dict(shapes=[(4096, 512)], rank=1, iters=4, mcr=2, dtype="f32"),
}


def _splitmix64(x: np.ndarray) -> np.ndarray:
    x = x + np.uint64(0x9E3779B97F4A7C15)
    z = x
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def hash_normal(seed: int, count: int, stream: int = 0) -> np.ndarray:
    """Deterministic N(0,1) float32 samples; ``(seed, stream)`` selects the sequence."""
    if count == 0:
        return np.zeros(0, dtype=np.float32)
    half = (count + 1) // 2
    base = (np.uint64(seed & 0xFFFFFFFF) << np.uint64(40)) ^ (
        np.uint64(stream & 0xFFFFFF) << np.uint64(16)
    )
    with np.errstate(over="ignore"):
        idx = np.arange(half, dtype=np.uint64) * np.uint64(2) + base * np.uint64(0x100000001B3)
        a = _splitmix64(idx)
        b = _splitmix64(idx + np.uint64(1))
    # 53-bit uniforms in (0, 1]
    u1 = ((a >> np.uint64(11)).astype(np.float64) + 1.0) * (1.0 / 9007199254740992.0)
    u2 = (b >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    r = np.sqrt(-2.0 * np.log(u1))
    z = np.empty(2 * half, dtype=np.float64)
    z[0::2] = r * np.cos(2 * np.pi * u2)
    z[1::2] = r * np.sin(2 * np.pi * u2)
    return z[:count].astype(np.float32)


def hash_tensors(shapes: List[Shape], seed: int) -> List[np.ndarray]:
    """One independent hash_normal stream per tensor."""
    return [
        hash_normal(seed, int(np.prod(s)) if len(s) else 1, stream=i).reshape(s)
        for i, s in enumerate(shapes)
    ]
