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

Bucket plumbing is native (include/psgd.h ``psgd_runs_*``): per DDP bucket layout a run table
(bucket offset, parameter, length: one run per parameter, 64-bit offsets) drives one HIP launch
that adds the bucket into the residual and, at completion, one that gathers the averages back
into the bucket buffer. No index maps, no full-size copy, no limit on the element count.

Because the residual lives in the state (not in ``p.grad``), the training loop zeroes
gradients as usual:

    state = PowerSGDState(Config(rank=2, num_iters_per_step=2, start_compressing_after_num_steps=0),
                          params=[p for p in model.parameters()])
    ddp_model.register_comm_hook(state, powersgd_hook)
    loss.backward(); optimizer.step(); optimizer.zero_grad()
"""
import ctypes
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from . import _lib
from .powersgd import Config, PowerSGD, _DTYPES, _psgd_host, _require_device, _stream


class _BucketRuns:
    """The run table of one DDP bucket layout (one run per parameter: bucket offset, parameter
    index, length), bound to device memory (psgd_runs_*)."""

    def __init__(self, key, buf: torch.Tensor, grads, idx, ntensors: int, code: int, dev_index: int):
        self.key = key
        esz = buf.element_size()
        self.offs = [(g.data_ptr() - buf.data_ptr()) // esz for g in grads]
        self.idx = list(idx)
        self.lens = [g.numel() for g in grads]
        self.runs = _lib.Runs(self.offs, self.idx, [0] * len(idx), self.lens, ntensors, code)
        self.ws = torch.empty(self.runs.workspace_bytes(), dtype=torch.uint8, device=buf.device)
        self.runs.bind(dev_index, self.ws.data_ptr())


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
        # the run-table kernels (psgd_runs_*) read buckets and write the residual at ONE element
        # size, the state's: a mixed-dtype parameter list would index them at the wrong width
        mixed = [i for i, p in enumerate(self.params) if p.dtype != p0.dtype]
        if mixed:
            raise RuntimeError(f"powersgd_hook needs one gradient dtype: parameter {mixed[0]} is "
                               f"{self.params[mixed[0]].dtype}, parameter 0 is {p0.dtype}")
        self._dev_index = _require_device(p0.device)
        self._code = _DTYPES[p0.dtype] if p0.dtype in _DTYPES else None
        if self._code is None:
            raise RuntimeError(f"powersgd_hook supports float32, bfloat16 and float64 gradients, got {p0.dtype}")
        self.residual = torch.zeros(numel, dtype=p0.dtype, device=p0.device)
        self.views: List[torch.Tensor] = []
        off = 0
        for p in self.params:
            self.views.append(self.residual[off:off + p.numel()].view(p.shape))
            off += p.numel()
        # per-parameter pointer tables (host arrays handed to psgd_runs_*): the residual views
        # (fixed) and the latest averaged outputs (refilled natively at every completion)
        self._res_ptrs = _lib.ptr_array([v.data_ptr() for v in self.views])
        self._out_ptrs = _lib.ptr_array([0] * len(self.views))
        # per DDP bucket index: the run table of its LATEST layout only (DDP rebuilds its buckets
        # after the first iteration; the old tables are dropped)
        self._runs: Dict[int, _BucketRuns] = {}
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
            if buf.dtype != self.residual.dtype:
                # DDP buckets carry the gradients' dtype; anything else (e.g. a bf16 bucket under
                # an fp32 state) would be read and written at the wrong element size
                raise RuntimeError(f"powersgd_hook: DDP bucket dtype {buf.dtype} differs from the state's "
                                   f"gradient dtype {self.residual.dtype}")
            runs = self._bucket_runs(bucket.index(), buf, grads, idx)
            self._ef_add(buf, runs)
            for i in idx:
                self._seen[i] = True
                self._nseen += 1
            self._pending.append((buf, runs, fut))
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

    def _bucket_runs(self, bucket_index: int, buf: torch.Tensor, grads, idx) -> _BucketRuns:
        """The bucket's run table (one run per parameter: bucket offset -> parameter, length),
        built once per bucket layout; only the bucket's latest layout is kept."""
        key = (buf.numel(), tuple(idx), tuple((g.data_ptr() - buf.data_ptr()) // buf.element_size() for g in grads))
        hit = self._runs.get(bucket_index)
        if hit is not None and hit.key == key:
            return hit
        self._runs.pop(bucket_index, None)
        r = self._new_runs(key, buf, grads, idx)
        self._runs[bucket_index] = r
        return r

    def _new_runs(self, key, buf, grads, idx) -> _BucketRuns:
        return _BucketRuns(key, buf, grads, idx, len(self.params), self._code, self._dev_index)

    def _ef_add(self, buf: torch.Tensor, runs: _BucketRuns) -> None:
        """Error feedback: residual += the bucket's fresh gradients, the whole bucket in one launch
        (autograd's accumulation into p.grad in the reference flow, README.md:39-42)."""
        runs.runs.add(buf.data_ptr(), ctypes.addressof(self._res_ptrs), _stream(buf.device))

    def _gather(self, pending, outs) -> None:
        """The averages, parameter by parameter, straight into each pending bucket's buffer (its
        own layout), one launch per bucket on the codec's stream."""
        _psgd_host.fill_list(outs, ctypes.addressof(self._out_ptrs), self._code, self._dev_index)
        stream = _stream(self.residual.device)
        for buf, runs, _ in pending:
            runs.runs.gather(buf.data_ptr(), ctypes.addressof(self._out_ptrs), stream)

    def _complete(self) -> None:
        outs = self.powersgd.aggregate(self.views)  # leaves the new residual in self.views
        pending, self._pending = self._pending, []
        self._seen = [False] * len(self.params)
        self._nseen = 0
        # the gathers read `outs` on the stream; the codec reuses its output buffer only at a later
        # aggregate (same stream) once no view of it is referenced: queued before that, safe
        self._gather(pending, outs)
        for buf, _, fut in pending:
            fut.set_result(buf)


def powersgd_hook(state: PowerSGDState, bucket: dist.GradBucket) -> torch.futures.Future[torch.Tensor]:
    """``DistributedDataParallel.register_comm_hook`` hook: the reference's PowerSGD flow."""
    return state._arrive(bucket)
