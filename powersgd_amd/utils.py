"""Helpers of the reference's ``powersgd/utils.py`` API (same names and behaviour).

These are the reference's generic utilities (pack/unpack with torch ops, distributed
detection, optimizer parameter listing). The hot path does not use ``pack``/``unpack``:
``AllReduce`` packs with the HIP flat kernel (include/psgd.h, psgd_flat_pack).
"""
from __future__ import annotations

from types import SimpleNamespace
from typing import List, Tuple

import torch


def pack(tensors: List[torch.Tensor]) -> Tuple[torch.Tensor, List[torch.Size]]:
    """One contiguous copy of ``tensors`` (reference utils.py:6-10)."""
    buffer = torch.cat([t.view(-1) for t in tensors])
    return buffer, [t.shape for t in tensors]


def unpack(buffer: torch.Tensor, shapes: List[torch.Size]) -> List[torch.Tensor]:
    """Views of the given shapes into a flat buffer (reference utils.py:13-22)."""
    out, idx = [], 0
    for s in shapes:
        end = idx + s.numel()
        out.append(buffer[idx:end].view(size=s))
        idx = end
    return out


def params_in_optimizer(optimizer: torch.optim.Optimizer) -> List[torch.Tensor]:
    """reference utils.py:25-29."""
    params: List[torch.Tensor] = []
    for group in optimizer.param_groups:
        params.extend(group["params"])
    return params


def is_distributed() -> bool:
    """reference utils.py:32-33."""
    return torch.distributed.is_available() and torch.distributed.is_initialized()


def flatten(tensors: List[List[torch.Tensor]]) -> List[torch.Tensor]:
    """reference utils.py:36-40."""
    out: List[torch.Tensor] = []
    for lst in tensors:
        out.extend(lst)
    return out


def allreduce_average(data, *args, **kwargs):
    """All-reduce average when torch.distributed is initialised, else nothing
    (reference utils.py:43-49)."""
    if is_distributed():
        data.div_(torch.distributed.get_world_size())
        return torch.distributed.all_reduce(data, *args, **kwargs)
    return SimpleNamespace(wait=lambda: None)
