"""PowerSGD aggregators — the reference's Python interface over the MI355X HIP codec.

Mirrors epfml/powersgd ``powersgd/powersgd.py`` (same class names, constructor
arguments, attributes, return values and in-place side effects):

* ``Aggregator``      reference :11-19
* ``AllReduce``       reference :22-31   (flat pack/scale/zero kernel + all-reduce)
* ``Config``          reference :34-38
* ``PowerSGD``        reference :41-105  (warm-up, compression mask, split/merge)
* ``BasicConfig``     reference :108-110
* ``BasicPowerSGD``   reference :113-275 (the hot path: libpsgd.so, see include/psgd.h)

Differences, all deliberate:
* Device tensors on a ROCm GPU only; the HIP library is mandatory (no CPU fallback).
* bfloat16 gradients are supported (the reference raises at its ``bmm``, :189): the
  gradient matrix is read/written in bf16, factors and arithmetic stay fp32.
* float64 gradients (the reference's own test dtype) run fp64 kernels with fp64 factors; as in
  the reference, torch's default dtype must then be float64 (P/Q follow it, :241-251).
* Returned compressed outputs are views of one flat buffer (allocated fresh per call)
  instead of separate ``empty_like`` tensors; uncompressed outputs are views in the
  reference too.
"""
from __future__ import annotations

import ctypes
import os
from abc import ABC, abstractmethod
from collections import defaultdict
from typing import Dict, List, NamedTuple, Optional, Sequence, Union

import torch

from . import _lib
from .utils import is_distributed

try:
    from . import _psgd_host  # native gradient split + pointer tables (csrc/psgd_host.cpp)
except ImportError as e:  # built together with libpsgd.so; no Python fallback
    raise _lib.LibraryMissing(
        "powersgd_amd/_psgd_host*.so not found: build it with "
        "`python -c 'import __graft_entry__ as g; g.build()'`"
    ) from e

_DTYPES = {torch.float32: _lib.PSGD_F32, torch.bfloat16: _lib.PSGD_BF16, torch.float64: _lib.PSGD_F64}


def _require_device(device: torch.device) -> int:
    if device.type != "cuda":
        raise RuntimeError(
            f"powersgd_amd runs its codec on MI355X GPUs (HIP); got tensors on '{device}'"
        )
    return device.index if device.index is not None else torch.cuda.current_device()


def _dtype_code(dtype: torch.dtype) -> int:
    try:
        return _DTYPES[dtype]
    except KeyError:
        raise RuntimeError(f"powersgd_amd supports float32, bfloat16 and float64 gradients, got {dtype}")


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _output_slab(shapes, code: int, dev_index: int):
    """Flat output buffer + per-tensor views (csrc/psgd_host.cpp OutputSlab): ``get()`` returns
    the views, handing the previous call's buffer out again only when no reference to any of
    its views survives anywhere (TensorImpl, PyObject and storage reference counts back at
    their creation values), else a fresh buffer, like the reference's per-call ``empty_like``
    (:153). ``flat`` is the buffer of the latest call.

    Outputs are produced on the codec's stream (torch's current stream). A consumer on ANOTHER
    stream must keep a reference to the outputs until its work is done (``record_stream`` alone
    does not delay the reuse here, unlike torch's caching allocator): the next step writes the
    buffer again once the last reference is dropped."""
    return _psgd_host.OutputSlab([list(s) for s in shapes], code, dev_index)


class Aggregator(ABC):
    """reference :11-19."""

    @abstractmethod
    def aggregate(self, gradients: List[torch.Tensor]) -> List[torch.Tensor]:
        """Average ``gradients`` across workers; mutates them (zero, or the compression error)."""


class AllReduce(Aggregator):
    """Flat all-reduce average of uncompressed tensors (reference :22-31).

    One HIP kernel copies every tensor (divided by the world size when distributed)
    into a flat buffer and zeroes the inputs; the flat buffer is SUM-all-reduced and
    the outputs are views of it, as in the reference.
    """

    def __init__(self):
        self._plans: Dict[tuple, "_FlatEntry"] = {}

    def aggregate(self, gradients: List[torch.Tensor]) -> List[torch.Tensor]:
        if len(gradients) == 0:
            return []
        g0 = gradients[0]
        dev_index = _require_device(g0.device)
        code = _dtype_code(g0.dtype)
        key = (tuple(g.shape for g in gradients), g0.dtype, dev_index)
        entry = self._plans.get(key)
        if entry is None:
            entry = self._plans[key] = _FlatEntry([g.shape for g in gradients], code, g0.dtype, g0.device)
        _psgd_host.fill_list(gradients, entry.ptr_addr, code, dev_index)
        return entry.run(entry.ptr_addr)


class _FlatEntry:
    """Flat-pack plan + workspace + pointer table + output slab of one tensor list."""

    def __init__(self, shapes, code: int, dtype, device):
        self.shapes = [torch.Size(s) for s in shapes]
        self.numel = sum(s.numel() for s in self.shapes)
        self.dtype, self.device = dtype, device
        self.plan = _lib.FlatPlan([s.numel() for s in self.shapes], code)
        self.ws = torch.empty(self.plan.workspace_bytes(), dtype=torch.uint8, device=device)
        self.plan.bind(device.index if device.index is not None else torch.cuda.current_device(),
                       self.ws.data_ptr())
        self.ptrs = _lib.ptr_array([0] * len(self.shapes))
        self.ptr_addr = ctypes.addressof(self.ptrs)
        self.slab = _output_slab(self.shapes, code, _require_device(device))

    def run(self, ptr_addr: int) -> List[torch.Tensor]:
        outs = self.slab.get()
        world = torch.distributed.get_world_size() if is_distributed() else 1
        self.plan.pack(ptr_addr, self.slab.data_ptr(), world, _stream(self.device))
        if is_distributed():
            torch.distributed.all_reduce(self.slab.flat[:self.numel])
        return outs


class Config(NamedTuple):
    """reference :34-38 (same fields and defaults)."""

    rank: int  # lower rank => more aggressive compression
    min_compression_rate: float = 2  # skip compression on some gradients
    num_iters_per_step: int = 1  # lower number => more aggressive compression
    start_compressing_after_num_steps: int = 100


class PowerSGD(Aggregator):
    """Applies PowerSGD only after a configurable number of steps, and only on
    parameters with strong compression (reference :41-105)."""

    def __init__(self, params: List[torch.Tensor], config: Config):
        self.config = config
        self.device = list(params)[0].device
        self.is_compressed_mask = [self._should_compress(p.shape) for p in params]
        self.step_counter = 0
        compressed_params, _ = self._split(params)
        self._powersgd = BasicPowerSGD(
            compressed_params,
            config=BasicConfig(rank=config.rank, num_iters_per_step=config.num_iters_per_step),
        )
        self._allreduce = AllReduce()
        # native split: one C++ pass checks every gradient and fills the compressed and
        # uncompressed pointer tables (reference _split :76-84 without Python lists)
        p = self._powersgd
        self._table = _psgd_host.PtrTable([list(t.shape) for t in params], self.is_compressed_mask,
                                          p._code, p._dev_index)
        unc_shapes = [t.shape for t, c in zip(params, self.is_compressed_mask) if not c]
        self._unc = _FlatEntry(unc_shapes, p._code, p.dtype, p.device) if unc_shapes else None
        # one fp32 collective can carry factor + uncompressed values (fp32 gradients only)
        self._merge_ok = p.dtype == torch.float32 and os.environ.get("PSGD_MERGE_ALLREDUCE", "1") != "0"
        # _merge order: position of tensor i in (compressed outputs + uncompressed outputs)
        nc = sum(self.is_compressed_mask)
        ic, iu, self._order = 0, nc, []
        for c in self.is_compressed_mask:
            self._order.append(ic if c else iu)
            ic, iu = (ic + 1, iu) if c else (ic, iu + 1)

    def aggregate(self, gradients: List[torch.Tensor]) -> List[torch.Tensor]:
        self.step_counter += 1
        if self.step_counter <= self.config.start_compressing_after_num_steps:
            return self._allreduce.aggregate(gradients)
        if not isinstance(gradients, list):
            gradients = list(gradients)
        self._table.fill(gradients)  # reference _split :76-84 + the checks its torch ops make
        codec = self._powersgd
        ipc = is_distributed() and codec._ipc_mode()
        comm = codec._rccl_comm() if is_distributed() and not ipc else None
        if ipc or comm is not None:
            # world size W, RCCL or the IPC exchange: the whole step in one library call on the
            # codec's stream; the uncompressed tensors (fp32) ride in the last factor's exchange
            u = self._unc
            if ipc:
                codec._ipc_setup(u.numel if u is not None and u.dtype == torch.float32 else 0)
            if u is not None and u.dtype == torch.float32:
                unc = u.slab.get()
                outs = codec._aggregate_table(self._table.comp_addr(),
                                              flat=(u.plan, self._table.unc_addr(), u.slab.data_ptr())) + unc
            else:
                outs = codec._aggregate_table(self._table.comp_addr())
                if u is not None:
                    outs = outs + u.run(self._table.unc_addr())
        elif self._unc is not None and is_distributed() and self._merge_ok:
            outs = self._aggregate_merged()
        elif self._unc is not None and not is_distributed():
            # world size 1: the uncompressed copy/zero rides in the codec's final launch
            u = self._unc
            unc = u.slab.get()
            outs = self._powersgd._aggregate_table(self._table.comp_addr(),
                                                   flat=(u.plan, self._table.unc_addr(), u.slab.data_ptr()))
            outs = outs + unc
        else:
            outs = self._powersgd._aggregate_table(self._table.comp_addr())
            if self._unc is not None:
                outs = outs + self._unc.run(self._table.unc_addr())
        return [outs[i] for i in self._order]  # reference _merge :86-99

    def close(self) -> None:
        """Collective: release the codec's multi-GPU transports (BasicPowerSGD.close)."""
        self._powersgd.close()

    def _aggregate_merged(self) -> List[torch.Tensor]:
        """World size > 1: ONE collective fewer per step. The uncompressed gradients
        (divided by W, reference utils.py:43-47) are packed behind the factor the last
        power iteration produces, and that iteration's SUM all-reduce (:204-209) carries
        both — on xGMI a sub-MB all-reduce costs its latency, not its bytes."""
        codec = self._powersgd
        if codec._p_comm is None:
            codec._attach_tail(self._unc.numel)
        comm = codec._last_comm()
        tail = comm[comm.numel() - self._unc.numel:]
        world = torch.distributed.get_world_size()
        self._unc.plan.pack(self._table.unc_addr(), tail.data_ptr(), world, _stream(self.device))
        outs = codec._aggregate_table(self._table.comp_addr(), last_comm=comm)
        unc = self._unc.slab.get()
        self._unc.slab.flat[:self._unc.numel].copy_(tail)
        return outs + unc

    def _split(self, params: List[torch.Tensor]):
        comp, unc = [], []
        for p, c in zip(params, self.is_compressed_mask):
            (comp if c else unc).append(p)
        return comp, unc

    def _merge(self, compressed: List[torch.Tensor], uncompressed: List[torch.Tensor]) -> List[torch.Tensor]:
        assert len(compressed) + len(uncompressed) == len(self.is_compressed_mask)
        ci, ui = iter(compressed), iter(uncompressed)
        return [next(ci) if c else next(ui) for c in self.is_compressed_mask]

    def _should_compress(self, shape: torch.Size) -> bool:
        return shape.numel() / avg_compressed_size(shape, self.config) > self.config.min_compression_rate


class BasicConfig(NamedTuple):
    """reference :108-110."""

    rank: int  # lower rank => more aggressive compression
    num_iters_per_step: int = 1  # lower number => more aggressive compression


class BasicPowerSGD(Aggregator):
    """PowerSGD codec on every given tensor (reference :113-275), on the HIP path.

    State matches the reference: ``_ps_buffer``/``_qs_buffer`` (fp32, group-ordered
    [B, n, r] / [B, m, r] batches) with views ``_ps``/``_qs``, ``step_counter``,
    ``generator`` (seeded 0 on the params' device and drawn exactly as the reference).
    """

    def __init__(self, params: List[torch.Tensor], config: BasicConfig):
        self.config = config
        self.params = list(params)
        self.device = self.params[0].device  # IndexError on an empty list, as the reference
        self.dtype = self.params[0].dtype
        self._dev_index = _require_device(self.device)
        self._code = _dtype_code(self.dtype)
        self.params_per_shape = self._matrices_per_shape(self.params)
        self._plan = _lib.Plan([tuple(p.shape) for p in self.params], config.rank,
                               config.num_iters_per_step, self._code)

        self.generator = torch.Generator(device=self.device).manual_seed(0)
        self.step_counter = 0
        p_batches = [self._init_p_batch(s, ps) for s, ps in self.params_per_shape.items()]
        q_batches = [self._init_q_batch(s, ps) for s, ps in self.params_per_shape.items()]
        self._ps_buffer = torch.cat([b.view(-1) for b in p_batches])
        self._qs_buffer = torch.cat([b.view(-1) for b in q_batches])
        self._ps = _views(self._ps_buffer, [b.shape for b in p_batches])
        self._qs = _views(self._qs_buffer, [b.shape for b in q_batches])
        pn, qn = self._plan.factor_numel()
        assert pn == self._ps_buffer.numel() and qn == self._qs_buffer.numel()
        # P/Q follow torch's default dtype, as in the reference (:241-251), whose bmm then needs
        # the gradients in that dtype (fp64 tests: torch.set_default_dtype(torch.float64),
        # tests/powersgd_test.py:38). bf16 gradients keep fp32 factors (the reference raises).
        want = torch.float64 if self.dtype == torch.float64 else torch.float32
        if self._ps_buffer.dtype != want:
            names = {torch.float64: "Double", torch.float32: "Float"}
            raise RuntimeError(f"expected scalar type {names[want]} but found "
                               f"{names.get(self._ps_buffer.dtype, self._ps_buffer.dtype)} (P/Q follow torch's "
                               f"default dtype; gradients are {self.dtype})")
        self._workspace = torch.empty(self._plan.workspace_bytes(), dtype=torch.uint8, device=self.device)
        self._plan.bind(self._dev_index, self._ps_buffer.data_ptr(), self._qs_buffer.data_ptr(),
                        self._workspace.data_ptr())
        self._out_numel = self._plan.output_numel()
        self._shapes = [p.shape for p in self.params]
        self._slab = _output_slab(self._shapes, self._code, self._dev_index)
        self._table = _psgd_host.PtrTable([list(s) for s in self._shapes], [True] * len(self._shapes),
                                          self._code, self._dev_index)
        self._p_comm: Optional[torch.Tensor] = None
        self._q_comm: Optional[torch.Tensor] = None
        self._buckets: Optional[List[tuple]] = None  # W > 1: (p_off, p_len, q_off, q_len) per bucket
        self._ipc_open = False  # W > 1 with PSGD_COMM=ipc: peers' exchange buffers mapped
        self._comm = None  # W > 1 over RCCL: the library's own communicator (_rccl_comm)

    def aggregate(self, gradients: List[torch.Tensor]) -> List[torch.Tensor]:
        """reference :146-235. Mutates ``gradients`` into the compression error."""
        if not isinstance(gradients, list):
            gradients = list(gradients)
        self._table.fill(gradients)  # dtype / device / shape / contiguity checks + pointers
        return self._aggregate_table(self._table.comp_addr())

    def _ipc_mode(self) -> bool:
        """PSGD_COMM=ipc (or PSGD_IPC_ALLREDUCE=1): every factor all-reduce of a step runs as a
        one-shot sum over IPC-mapped exchange buffers with device-side flags (psgd_aggregate_ipc;
        one node, one process per GPU). fp32/bf16 plans; any torch.distributed backend carries
        the one-off handle exchange."""
        mode = os.environ.get("PSGD_COMM", "rccl")
        if os.environ.get("PSGD_IPC_ALLREDUCE") == "1":
            mode = "ipc"
        return mode == "ipc" and self.dtype != torch.float64

    def _ipc_setup(self, flat_numel: int = 0) -> None:
        """Collective, once: create this rank's exchange buffer (room for ``flat_numel``
        uncompressed values), all-gather the IPC handles and open the peers' buffers."""
        if self._ipc_open:
            return
        dist = torch.distributed
        world = dist.get_world_size()
        handle = self._plan.ipc_create(flat_numel)
        handles: List = [None] * world
        dist.all_gather_object(handles, handle)
        err = None
        try:
            self._plan.ipc_open(world, dist.get_rank(), handles)
        except RuntimeError as e:
            err = str(e)
        # collective outcome: one rank failing to map a peer must not leave the others polling
        # flags it will never raise
        errs: List = [None] * world
        dist.all_gather_object(errs, err)
        bad = [(r, e) for r, e in enumerate(errs) if e is not None]
        if bad:
            if err is None:
                self._plan.ipc_close()
            raise RuntimeError(f"IPC exchange setup failed on rank(s) {bad}")
        # the teardown barrier runs on a group of its own (CPU, gloo): at an uneven exit it can
        # only meet other ranks' teardown barriers, never pair with a gradient collective of the
        # default group
        self._ipc_group = dist.new_group(backend="gloo")
        self._ipc_open = True
        _register_exit_close(self)

    def ipc_status(self) -> bool:
        """True if a device-side exchange wait has timed out since the exchange was set up
        (synchronous; sticky until ``close_ipc``). Steps enqueued after a timed-out wait return
        NaN sums, and the next ``aggregate`` call raises."""
        return self._ipc_open and self._plan.ipc_status()

    def close_ipc(self, timeout: Optional[float] = None) -> None:
        """Collective teardown of the IPC exchange session: end it (the peer mappings stay with
        the process's exchange arena), then a barrier on the exchange's own gloo group, so that
        no rank re-zeroes its region for a new session (or hands it to another codec) while a
        peer's exchange kernel may still read it (include/psgd.h). Every rank must call it
        (``close()`` does), or leave it to the exit hook. ``timeout`` (seconds) bounds the barrier (the exit hook uses it: a rank
        that died must not hang the others at exit)."""
        if self._ipc_open:
            self._plan.ipc_close()
            self._ipc_open = False
            group = getattr(self, "_ipc_group", None)
            if timeout is None:
                torch.distributed.barrier(group=group)
            else:
                import datetime

                torch.distributed.barrier(group=group, async_op=True).wait(datetime.timedelta(seconds=timeout))
            self._ipc_group = None

    def close(self) -> None:
        """Release the multi-GPU transports (collective: every rank calls it). The exchange
        buffers of PSGD_COMM=ipc are unmapped and the ranks meet at a barrier before any frees
        its buffer; without this call an exit hook does the same with a bounded barrier."""
        self.close_ipc()
        self._comm = None

    def _rccl_comm(self) -> Optional["_lib.Comm"]:
        """World size > 1 on the NCCL (RCCL) backend: a communicator the library drives itself on
        the codec's stream (psgd_comm_init; the id travels over the default process group), so a
        whole step is one call (psgd_aggregate_comm). None on gloo, for fp64 plans, with
        PSGD_COMM=torch (the torch.distributed path below) or PSGD_COMM=ipc."""
        if self._comm is None:
            self._comm = False
            dist = torch.distributed
            if (os.environ.get("PSGD_COMM", "rccl") == "rccl" and dist.get_backend() == "nccl"
                    and self.dtype != torch.float64 and not self._ipc_mode()):
                world, rank = dist.get_world_size(), dist.get_rank()
                obj = [_lib.comm_unique_id() if rank == 0 else None]
                dist.broadcast_object_list(obj, src=0)
                self._comm = _lib.Comm(world, rank, obj[0], self._dev_index)
        return self._comm or None

    def _attach_tail(self, numel: int) -> None:
        """Re-home the P and Q state buffers at the head of [factor | tail] allocations so
        that the last all-reduce of a step can carry ``numel`` more fp32 values (the
        uncompressed gradients, see PowerSGD._aggregate_merged). State values are kept."""
        pn, qn = self._ps_buffer.numel(), self._qs_buffer.numel()
        self._p_comm = torch.zeros(pn + numel, dtype=torch.float32, device=self.device)
        self._q_comm = torch.zeros(qn + numel, dtype=torch.float32, device=self.device)
        self._p_comm[:pn].copy_(self._ps_buffer)
        self._q_comm[:qn].copy_(self._qs_buffer)
        self._ps_buffer = self._p_comm[:pn]
        self._qs_buffer = self._q_comm[:qn]
        self._ps = _views(self._ps_buffer, [p.shape for p in self._ps])
        self._qs = _views(self._qs_buffer, [q.shape for q in self._qs])
        self._plan.bind(self._dev_index, self._ps_buffer.data_ptr(), self._qs_buffer.data_ptr(),
                        self._workspace.data_ptr())

    def _last_comm(self) -> torch.Tensor:
        """[factor | tail] buffer whose factor the last iteration of this step produces."""
        last = self.config.num_iters_per_step - 1
        return self._q_comm if self._plan.out_factor(self.step_counter, last) == 0 else self._p_comm

    def _aggregate_table(self, ptrs: int, last_comm: Optional[torch.Tensor] = None,
                         flat: Optional[tuple] = None) -> List[torch.Tensor]:
        """The codec on a native pointer table (address of ``void*[len(params)]``).
        ``last_comm``: all-reduce this [factor | tail] buffer in place of the last factor.
        ``flat``: (FlatPlan, uncompressed pointer table, flat output pointer) packed in the
        same final launch (world size 1, psgd_aggregate_flat)."""
        outs = self._slab.get()
        out_ptr = self._slab.data_ptr()
        stream = _stream(self.device)
        step = self.step_counter
        ipc = is_distributed() and last_comm is None and self._ipc_mode()
        comm = self._rccl_comm() if is_distributed() and last_comm is None and not ipc else None
        if ipc:
            self._ipc_setup(0)
            f = flat if flat is not None else (None, None, 0)
            self._plan.aggregate_ipc(ptrs, out_ptr, step, f[0], f[1], f[2], stream)
        elif comm is not None:
            f = flat if flat is not None else (None, None, 0)
            self._plan.aggregate_comm(ptrs, out_ptr, step, f[0], f[1], f[2], comm, stream)
        elif is_distributed():
            world = torch.distributed.get_world_size()
            iters = self.config.num_iters_per_step
            if self._buckets is None:
                self._setup_buckets()
            if len(self._buckets) > 1:
                self._aggregate_buckets(ptrs, out_ptr, step, world, stream, last_comm)
            else:
                for it in range(iters):
                    self._plan.compress(ptrs, step, it, stream)
                    buf = self._qs_buffer if self._plan.out_factor(step, it) == 0 else self._ps_buffer
                    if it == iters - 1 and last_comm is not None:
                        buf = last_comm
                    torch.distributed.all_reduce(buf)  # SUM of the local factors, reference :207
                self._plan.decompress(ptrs, out_ptr, step, world, stream)
        elif flat is not None:
            self._plan.aggregate_flat(ptrs, out_ptr, step, flat[0], flat[1], flat[2], stream)
        else:
            self._plan.aggregate(ptrs, out_ptr, step, stream)
        self.step_counter += 1
        return outs

    def _setup_buckets(self, want: Optional[int] = None) -> None:
        """Cut the shape groups into up to PSGD_BUCKETS (default 4) consecutive buckets of about
        equal gradient size. Each iteration's factor all-reduce (reference :204-209) is then
        issued per bucket slice, asynchronously, right after that bucket's kernels: bucket b's
        collective overlaps bucket b+1's product (RCCL runs on its own stream), and the next
        iteration of bucket b waits only for bucket b's collective. SUM over slices == SUM over
        the whole buffer, element by element. fp64 plans and PSGD_BUCKETS=1 keep one collective."""
        if want is None:
            want = int(os.environ.get("PSGD_BUCKETS", "4"))
        groups = self._plan.groups()
        if self.dtype == torch.float64 or want <= 1 or len(groups) < 2:
            self._buckets = [(0, self._ps_buffer.numel(), 0, self._qs_buffer.numel())]
            return
        cost = [c * n * m for n, m, _r, c in groups]
        total, nb = float(sum(cost)), min(want, len(groups))
        ends, acc = [], 0.0
        for g, c in enumerate(cost):
            acc += c
            left_groups, left_buckets = len(groups) - g - 1, nb - len(ends) - 1
            if len(ends) < nb - 1 and (acc >= total * (len(ends) + 1) / nb or left_groups == left_buckets):
                ends.append(g + 1)
        ends.append(len(groups))
        self._plan.set_buckets(ends)
        self._buckets = [self._plan.bucket_range(b) for b in range(len(ends))]

    def _aggregate_buckets(self, ptrs: int, out_ptr: int, step: int, world: int, stream: int,
                           last_comm: Optional[torch.Tensor]) -> None:
        iters = self.config.num_iters_per_step
        nb = len(self._buckets)
        works: List = [None] * nb
        for it in range(iters):
            which = self._plan.out_factor(step, it)
            state = self._qs_buffer if which == 0 else self._ps_buffer
            comm = last_comm if (it == iters - 1 and last_comm is not None) else None
            for b, (po, pl, qo, ql) in enumerate(self._buckets):
                if works[b] is not None:
                    works[b].wait()  # this bucket's previous collective (stream-ordered under RCCL)
                self._plan.compress_bucket(ptrs, step, it, b, stream)
                off, ln = (qo, ql) if which == 0 else (po, pl)
                if comm is None:
                    buf = state[off:off + ln]
                else:  # [factor | uncompressed tail]: the last bucket's slice carries the tail
                    buf = comm[off:] if b == nb - 1 else comm[off:off + ln]
                works[b] = torch.distributed.all_reduce(buf, async_op=True)  # SUM, reference :207
        for b in range(nb):
            works[b].wait()
            self._plan.decompress_bucket(ptrs, out_ptr, step, world, b, stream)

    def _init_p_batch(self, shape: torch.Size, params: List[torch.Tensor]) -> torch.Tensor:
        rank = min(self.config.rank, min(shape))
        return torch.randn([len(params), shape[0], rank], generator=self.generator, device=self.device)

    def _init_q_batch(self, shape: torch.Size, params: List[torch.Tensor]) -> torch.Tensor:
        rank = min(self.config.rank, min(shape))
        return torch.randn([len(params), shape[1], rank], generator=self.generator, device=self.device)

    @classmethod
    def _matrices_per_shape(cls, tensors: List[torch.Tensor]) -> Dict[torch.Size, List[torch.Tensor]]:
        shape2tensors: Dict[torch.Size, List[torch.Tensor]] = defaultdict(list)
        for t in tensors:
            m = view_as_matrix(t)
            shape2tensors[m.shape].append(m)
        return shape2tensors

    @property
    def uncompressed_num_floats(self) -> int:
        return sum(p.shape.numel() for p in self.params)

    @property
    def compressed_num_floats(self) -> float:
        return sum(avg_compressed_size(p.shape, self.config) for p in self.params)

    @property
    def compression_rate(self) -> float:
        return self.uncompressed_num_floats / self.compressed_num_floats


_EXIT_CLOSE: "weakref.WeakSet" = None


def _register_exit_close(codec: "BasicPowerSGD") -> None:
    """At interpreter exit, close every still-open IPC exchange (bounded barrier on the
    exchange's own gloo group, never the default group), so that a rank that finishes first does
    not free an exchange buffer a slower peer's last exchange kernel may still read (the peers
    unmap before anyone frees). Explicit ``close()`` on every rank is the documented teardown."""
    global _EXIT_CLOSE
    if _EXIT_CLOSE is None:
        import atexit
        import weakref

        _EXIT_CLOSE = weakref.WeakSet()

        def _close_all():
            for c in list(_EXIT_CLOSE):
                try:
                    if c._ipc_open and torch.distributed.is_initialized():
                        c.close_ipc(timeout=float(os.environ.get("PSGD_IPC_EXIT_TIMEOUT", "30")))
                except Exception:  # exit path: never raise
                    pass

        atexit.register(_close_all)
    _EXIT_CLOSE.add(codec)


def _views(buf: torch.Tensor, shapes) -> List[torch.Tensor]:
    out, i = [], 0
    for s in shapes:
        n = s.numel()
        out.append(buf[i:i + n].view(s))
        i += n
    return out


def batch_transpose(batch_of_matrices: torch.Tensor) -> torch.Tensor:
    """reference :279-280."""
    return batch_of_matrices.permute([0, 2, 1])


def view_as_matrix(tensor: torch.Tensor) -> torch.Tensor:
    """[output features, input features (x kernel dims)] view (reference :283-289)."""
    return tensor.view(tensor.shape[0], -1)


def avg_compressed_size(shape: torch.Size, config: Union[Config, BasicConfig]) -> float:
    """reference :292-294 — on the ORIGINAL tensor shape."""
    rank = min(config.rank, min(shape))
    return 0.5 * config.num_iters_per_step * rank * sum(shape)
