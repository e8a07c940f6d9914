"""DistributedDataParallel communication hook running this package's PowerSGD codec.

The reference drives PowerSGD from the optimizer (``optimizer_step``, powersgd/__init__.py:
7-25): ONE ``PowerSGD`` over all parameters in optimizer order, the error-feedback residual
kept in ``p.grad`` so the next backward adds onto it (README.md:39-42). Under
``DistributedDataParallel`` the gradients reach the aggregator bucket by bucket through
``register_comm_hook`` (the paper code plugs PowerSGD in that way, paper-code/
train_pytorch.py:106-131). This adapter reproduces the reference flow exactly, independent of
how DDP buckets the parameters (and of its bucket rebuild after the first iteration):

* the state owns one ``PowerSGD`` over ``params`` in the given (optimizer) order — the same
  compression mask, shape-group batching, P/Q state and step counter as the reference's
  ``PowerSGD(params, config)`` (reference :41-105, :113-275);
* it owns the error-feedback residual per parameter (one flat buffer): each bucket's fresh
  gradients are ADDED to their parameters' residual (what autograd's accumulation into
  ``p.grad`` does in the reference flow);
* a bucket's future completes when the LAST bucket of the iteration has arrived: then one
  ``aggregate`` runs over all parameters (its factor all-reduces on the default process group,
  reference :207) and every pending bucket receives its averaged approximation in its own
  layout. DDP waits on all bucket futures only after backward has launched every hook, so the
  deferral is legal; it trades DDP's per-bucket overlap for the reference's exact semantics.

Because the residual lives in the state (not in ``p.grad``), the training loop zeroes
gradients as usual:

    state = PowerSGDState(Config(rank=2, num_iters_per_step=2, start_compressing_after_num_steps=0),
                          params=[p for p in model.parameters()])
    ddp_model.register_comm_hook(state, powersgd_hook)
    loss.backward(); optimizer.step(); optimizer.zero_grad()
"""
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from .powersgd import Config, PowerSGD


class PowerSGDState:
    """Hook state: one codec + residual buffer over ``params`` (the optimizer's order)."""

    def __init__(self, config: Config, params, process_group=None):
        if process_group is not None and process_group is not dist.group.WORLD:
            raise ValueError("powersgd_hook all-reduces on the default process group (reference :207)")
        self.config = config
        self.params: List[torch.nn.Parameter] = [p for p in params if p.requires_grad]
        if not self.params:
            raise IndexError("list index out of range")  # the reference's PowerSGD on []
        self._index: Dict[int, int] = {id(p): i for i, p in enumerate(self.params)}
        numel = sum(p.numel() for p in self.params)
        p0 = self.params[0]
        self.residual = torch.zeros(numel, dtype=p0.dtype, device=p0.device)
        self.views: List[torch.Tensor] = []
        self._offs: List[int] = []
        off = 0
        for p in self.params:
            self._offs.append(off)
            self.views.append(self.residual[off:off + p.numel()].view(p.shape))
            off += p.numel()
        # per DDP bucket index: (layout key, int32 device index map) of its LATEST layout only
        # (DDP rebuilds its buckets after the first iteration; the old maps are dropped)
        self._gidx: Dict[int, tuple] = {}
        self.powersgd = PowerSGD(self.views, config)
        self._seen = [False] * len(self.params)
        self._nseen = 0
        self._pending: List[tuple] = []

    def _arrive(self, bucket: "dist.GradBucket") -> "torch.futures.Future[torch.Tensor]":
        fut: torch.futures.Future = torch.futures.Future()
        try:
            params, grads = bucket.parameters(), bucket.gradients()
            idx = []
            for p, g in zip(params, grads):
                i = self._index.get(id(p))
                if i is None:
                    raise RuntimeError("DDP bucket holds a parameter that PowerSGDState was not given")
                if self._seen[i]:
                    raise RuntimeError("parameter reached powersgd_hook twice in one iteration")
                idx.append(i)
            buf = bucket.buffer()
            gidx = self._gather_index(bucket.index(), buf, grads, idx)
            # error feedback: residual + fresh gradient, the whole bucket in one indexed add
            # (bucket buffer position -> residual position; every position once)
            self.residual.index_add_(0, gidx, buf)
            for i in idx:
                self._seen[i] = True
                self._nseen += 1
            self._pending.append((buf, gidx, fut))
            if self._nseen == len(self.params):
                self._complete()
            elif bucket.is_last():
                # DDP's last bucket arrived but some trainable parameter never did (e.g. one
                # DDP ignores): no aggregate can run, and waiting would hang DDP's backward
                missing = [i for i, s in enumerate(self._seen) if not s]
                raise RuntimeError(f"powersgd_hook: {len(missing)} parameter(s) given to PowerSGDState never "
                                   f"reached a DDP bucket (first index {missing[0]}); give the state exactly "
                                   "the parameters DDP reduces")
        except Exception as e:
            self._fail(e, fut)
            raise
        return fut

    def _fail(self, err: Exception, fut: "torch.futures.Future") -> None:
        """Fail this iteration: every pending bucket future (and this one) gets the exception, so
        DDP's wait raises instead of hanging, and the next iteration starts clean."""
        pending, self._pending = self._pending, []
        self._seen = [False] * len(self.params)
        self._nseen = 0
        for *_, f in pending:
            if not f.done():
                f.set_exception(err)
        if not fut.done():
            fut.set_exception(err)

    def _gather_index(self, bucket_index: int, buf: torch.Tensor, grads, idx) -> torch.Tensor:
        """Device index: position k of the bucket's flat buffer -> its position in the state's
        flat residual. int32 (4 bytes per gradient element: index_add_ / index_select take it),
        built once per bucket layout; only the bucket's latest layout is kept."""
        key = (buf.numel(), tuple(idx), tuple((g.data_ptr() - buf.data_ptr()) // buf.element_size() for g in grads))
        hit = self._gidx.get(bucket_index)
        if hit is not None and hit[0] == key:
            return hit[1]
        if self.residual.numel() >= 2 ** 31:
            raise RuntimeError("powersgd_hook: more than 2^31 gradient elements (int32 index maps)")
        host = torch.empty(buf.numel(), dtype=torch.int32)
        for g, i in zip(grads, idx):
            off = (g.data_ptr() - buf.data_ptr()) // buf.element_size()
            host[off:off + g.numel()] = torch.arange(self._offs[i], self._offs[i] + g.numel(), dtype=torch.int32)
        self._gidx.pop(bucket_index, None)  # free the stale layout's map before the new upload
        gidx = host.to(buf.device)
        self._gidx[bucket_index] = (key, gidx)
        return gidx

    def _complete(self) -> None:
        outs = self.powersgd.aggregate(self.views)  # leaves the new residual in self.views
        pending, self._pending = self._pending, []
        self._seen = [False] * len(self.params)
        self._nseen = 0
        # the averages in the state's order (a transient copy: the compressed and uncompressed
        # outputs live in two buffers), then one gather per bucket, in its layout
        flat = torch.cat([o.reshape(-1) for o in outs])
        for buf, gidx, fut in pending:
            fut.set_result(flat.index_select(0, gidx))
        del flat


def powersgd_hook(state: PowerSGDState, bucket: dist.GradBucket) -> torch.futures.Future[torch.Tensor]:
    """``DistributedDataParallel.register_comm_hook`` hook: the reference's PowerSGD flow."""
    return state._arrive(bucket)
