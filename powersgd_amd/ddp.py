"""DistributedDataParallel communication hook running this package's PowerSGD codec.

The reference drives PowerSGD from the optimizer (``optimizer_step``, powersgd/__init__.py:
7-25) and keeps the error-feedback residual in ``p.grad``, so the next backward adds onto it.
Under ``DistributedDataParallel`` the gradients reach the aggregator as buckets through
``register_comm_hook`` (the paper code compares against the upstream hook that way,
SURVEY.md §8(f) row 3). This adapter keeps the reference's algorithm and semantics per bucket:

* one ``PowerSGD`` per bucket layout (shapes + dtype), i.e. the same warm-up, compression mask,
  shape-group batching, P/Q state and step counter as the reference applied to that bucket's
  gradients (reference :41-105, :113-275);
* error feedback exactly as the reference gets it through autograd accumulation: the stored
  residual is added to the fresh bucket gradients before the codec runs (README.md:39-42),
  and the codec leaves the new residual in that buffer;
* the averaged approximation (plus the uncompressed averages) is returned to DDP, which
  writes it into ``p.grad`` for the optimizer.

The factor all-reduces use the default process group, like the reference (:207).

    from powersgd_amd import Config
    from powersgd_amd.ddp import PowerSGDState, powersgd_hook
    ddp_model.register_comm_hook(PowerSGDState(Config(rank=1, num_iters_per_step=2,
                                                      start_compressing_after_num_steps=0)),
                                 powersgd_hook)
"""
from typing import Dict, Tuple

import torch
import torch.distributed as dist

from .powersgd import Config, PowerSGD


class PowerSGDState:
    """Hook state: one codec + residual (error-feedback) buffer per SET of bucket parameters.

    Keyed by the parameters rather than the bucket layout: DDP rebuilds its buckets after the
    first iteration (new order inside a bucket), and the residual and P/Q state must follow
    the parameters through that. The codec batches the parameters in the order the set was
    first seen."""

    def __init__(self, config: Config, process_group=None):
        if process_group is not None and process_group is not dist.group.WORLD:
            raise ValueError("powersgd_hook all-reduces on the default process group (reference :207)")
        self.config = config
        self._sets: Dict[frozenset, dict] = {}

    def _entry(self, params) -> dict:
        key = frozenset(id(p) for p in params)
        e = self._sets.get(key)
        if e is None:
            numel = sum(p.numel() for p in params)
            resid = torch.zeros(numel, dtype=params[0].dtype, device=params[0].device)
            views, off = [], 0
            for p in params:
                views.append(resid[off:off + p.numel()].view(p.shape))
                off += p.numel()
            e = {"ids": [id(p) for p in params], "resid": resid, "views": views,
                 "psgd": PowerSGD(views, self.config)}
            self._sets[key] = e
        return e


def powersgd_hook(state: PowerSGDState, bucket: dist.GradBucket) -> torch.futures.Future[torch.Tensor]:
    """``DistributedDataParallel.register_comm_hook`` hook: PowerSGD on one gradient bucket."""
    params = bucket.parameters()
    grads = bucket.gradients()
    e = state._entry(params)
    slot = {id(p): g for p, g in zip(params, grads)}
    # error feedback: residual += fresh gradients (what autograd accumulation does to the
    # reference's p.grad); the codec then leaves the new residual in the same buffer
    for pid, r in zip(e["ids"], e["views"]):
        r.add_(slot[pid])
    outs = e["psgd"].aggregate(e["views"])
    # the averaged gradients go back in the bucket's own layout
    buf = bucket.buffer()
    out = torch.empty_like(buf)
    for pid, o in zip(e["ids"], outs):
        g = slot[pid]
        off = (g.data_ptr() - buf.data_ptr()) // buf.element_size()
        out[off:off + g.numel()].view(g.shape).copy_(o)
    fut: torch.futures.Future[torch.Tensor] = torch.futures.Future()
    fut.set_result(out)
    return fut
