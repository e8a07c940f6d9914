"""Host-memory PowerSGD: gradients that live in CPU memory (a CPU-run model), compressed and
decompressed on one or more MI355X GPUs.

The reference runs PowerSGD where the gradients are (``PowerSGD.aggregate``, reference
powersgd/powersgd.py:64-74, fed by ``optimizer_step``, powersgd/__init__.py:7-25). For a
model that runs on the CPU, this class keeps that exact contract — CPU tensors in, CPU
tensors out, the caller's gradients overwritten with the error-feedback residual — and runs
the codec on the GPUs:

* **Layout.** Compressed tensors are grouped by matrix shape (the reference's batching,
  :253-263) and the groups are bin-packed (longest processing time first) into
  ``len(devices) x chunks`` bins. Shape groups are never split: at rank 1 a group shares ONE
  joint norm (orthogonalization.py:5-6), so whole groups keep world-size-1 semantics with no
  cross-GPU traffic ("single-source sharded").
* **Pipeline.** Per device, three HIP streams: host-to-device copies of bin c+1 overlap the
  codec of bin c, which overlaps the device-to-host copies (outputs and residuals) of bin
  c-1. PCIe is full duplex, so the inbound and outbound traffic overlap too.
* **Pinned gradients.** ``pin_gradients()`` re-homes every ``p.grad`` as a view of ONE pinned
  host buffer laid out bin by bin, so each bin moves with one DMA per direction and autograd
  keeps accumulating into it. Unpinned gradients work too (staged through that buffer with a
  CPU copy each way).
* **State.** P/Q start from the reference's own initialisation (``torch.Generator`` on the
  parameters' device — here the CPU — seeded 0, every P batch then every Q batch, :123-144),
  scattered to the bins, so results equal the single-process reference (tests/test_gpu_host.py).
* Uncompressed tensors never leave the host: at world size 1 ``AllReduce`` is a copy plus a
  zero (:22-31, utils.py:43-49).
* ``residual="device"`` (opt-in semantic variant): the error-feedback residual of the
  compressed tensors stays on the GPU between steps and only the outputs return over PCIe
  (half the outbound bytes). Each ``aggregate`` then takes the FRESH gradients (the caller
  zeroes ``p.grad`` every step, e.g. ``optimizer.zero_grad()``, as with the DDP hook) and adds
  them to the device residual on the GPU — the same single add autograd's accumulation into
  ``p.grad`` performs in the reference flow (README.md:39-42), so the numbers are identical; the
  compressed inputs are zeroed (consumed) instead of being overwritten with the residual, so a
  caller that skips ``zero_grad()`` still hands only fresh gradients to the next step.
  ``residual()`` copies the device residual back on demand.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Optional, Sequence

import torch

from .powersgd import BasicConfig, BasicPowerSGD, Config, avg_compressed_size
from .utils import is_distributed


class HostPowerSGD:
    """Drop-in for ``powersgd.PowerSGD`` on CPU parameters (world size 1)."""

    def __init__(self, params: List[torch.Tensor], config: Config, devices: Optional[Sequence[int]] = None,
                 chunks: int = 2, residual: str = "host"):
        params = list(params)
        if residual not in ("host", "device"):
            raise ValueError("residual must be 'host' (the reference's contract) or 'device'")
        self.residual_on_device = residual == "device"
        if is_distributed():
            # world-size-1 semantics only: the factors of every bin would be all-reduced while
            # the uncompressed and warm-up paths stay local (a mix of global and local means)
            raise RuntimeError("HostPowerSGD serves one process (world size 1); with a process group "
                               "use PowerSGD on GPU-resident gradients, one rank per GPU")
        self.config = config
        self.device = params[0].device  # as the reference: the parameters' device (CPU here)
        if self.device.type != "cpu":
            raise RuntimeError("HostPowerSGD takes CPU parameters; use PowerSGD for GPU-resident ones")
        self.dtype = params[0].dtype
        self.is_compressed_mask = [
            p.shape.numel() / avg_compressed_size(p.shape, config) > config.min_compression_rate for p in params
        ]
        self.step_counter = 0
        self.shapes = [p.shape for p in params]
        devices = list(devices) if devices is not None else list(range(torch.cuda.device_count()))
        if not devices:
            raise RuntimeError("HostPowerSGD needs at least one GPU")
        comp = [i for i, c in enumerate(self.is_compressed_mask) if c]
        if not comp:
            raise IndexError("list index out of range")  # the reference's BasicPowerSGD on []
        self.unc = [i for i, c in enumerate(self.is_compressed_mask) if not c]

        # shape groups in first-appearance order (reference :253-263) and their init state
        groups: "OrderedDict[tuple, List[int]]" = OrderedDict()
        for i in comp:
            n = self.shapes[i][0]
            groups.setdefault((n, self.shapes[i].numel() // n), []).append(i)
        gen = torch.Generator(device="cpu").manual_seed(0)  # reference :123 (CPU params)
        rk = {k: min(config.rank, min(k)) for k in groups}
        p0 = {k: torch.randn([len(v), k[0], rk[k]], generator=gen) for k, v in groups.items()}
        q0 = {k: torch.randn([len(v), k[1], rk[k]], generator=gen) for k, v in groups.items()}

        # longest-processing-time packing of whole groups into devices x chunks bins
        nbins = len(devices) * max(1, int(chunks))
        load = [0] * nbins
        members: List[List[tuple]] = [[] for _ in range(nbins)]
        for key in sorted(groups, key=lambda k: -len(groups[k]) * k[0] * k[1]):
            b = min(range(nbins), key=lambda j: load[j])
            members[b].append(key)
            load[b] += len(groups[key]) * key[0] * key[1]
        order = list(groups)  # keep the global group order inside a bin
        self.bins = []
        for b in range(nbins):
            keys = sorted(members[b], key=order.index)
            if not keys:
                continue
            idx = [i for k in keys for i in groups[k]]
            idx.sort()  # tensor order inside the bin: groups keep first-appearance order
            self.bins.append({"dev": devices[b % len(devices)], "idx": idx, "keys": keys})

        # host layout: bins back to back, then the uncompressed tensors
        self.offsets: Dict[int, int] = {}
        off = 0
        for bn in self.bins:
            bn["lo"] = off
            for i in bn["idx"]:
                self.offsets[i] = off
                off += self.shapes[i].numel()
            bn["hi"] = off
        for i in self.unc:
            self.offsets[i] = off
            off += self.shapes[i].numel()
        self.numel = off
        self.host_grads = torch.zeros(self.numel, dtype=self.dtype).pin_memory()

        # per bin: device buffer, codec, streams; the codec's state comes from the host init
        self.streams: Dict[int, tuple] = {}
        for bn in self.bins:
            dev = torch.device("cuda", bn["dev"])
            if bn["dev"] not in self.streams:
                with torch.cuda.device(dev):
                    self.streams[bn["dev"]] = (torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev))
            with torch.cuda.device(dev):
                bn["dflat"] = torch.zeros(bn["hi"] - bn["lo"], dtype=self.dtype, device=dev)
                if self.residual_on_device:  # the fresh gradients land here, then add into dflat
                    bn["dstage"] = torch.zeros(bn["hi"] - bn["lo"], dtype=self.dtype, device=dev)
                bn["dgrads"] = [self._view(bn["dflat"], i, base=bn["lo"]) for i in bn["idx"]]
                codec = BasicPowerSGD(bn["dgrads"], BasicConfig(config.rank, config.num_iters_per_step))
                codec._ps_buffer.copy_(torch.cat([p0[k].reshape(-1) for k in bn["keys"]]))
                codec._qs_buffer.copy_(torch.cat([q0[k].reshape(-1) for k in bn["keys"]]))
                bn["codec"] = codec
                bn["events"] = [torch.cuda.Event(), torch.cuda.Event()]

    def _new_outputs(self) -> None:
        """Fresh pinned outputs every step, as the reference returns fresh tensors (a caller
        may hold last step's outputs). torch's caching host allocator recycles the block of
        an output nobody holds any more once its copies have completed."""
        self.host_out = torch.empty(self.numel, dtype=self.dtype, pin_memory=True)
        self._out_views = [self._view(self.host_out, i) for i in range(len(self.shapes))]

    def _view(self, flat: torch.Tensor, i: int, base: int = 0) -> torch.Tensor:
        o = self.offsets[i] - base
        return flat[o:o + self.shapes[i].numel()].view(self.shapes[i])

    def pin_gradients(self, params: List[torch.Tensor]) -> None:
        """Make every ``p.grad`` a view of the pinned, bin-ordered host buffer (current values
        kept); autograd then accumulates straight into DMA-able memory."""
        for i, p in enumerate(params):
            v = self._view(self.host_grads, i)
            if p.grad is not None:
                v.copy_(p.grad)
            else:
                v.zero_()
            p.grad = v

    def _pinned_in_place(self, gradients: List[torch.Tensor]) -> bool:
        return all(g.data_ptr() == self._view(self.host_grads, i).data_ptr() for i, g in enumerate(gradients))

    def aggregate(self, gradients: List[torch.Tensor]) -> List[torch.Tensor]:
        """reference PowerSGD.aggregate (:64-74) on CPU tensors; mutates ``gradients``."""
        gradients = list(gradients)
        if len(gradients) != len(self.shapes):
            raise ValueError(f"expected {len(self.shapes)} gradients, got {len(gradients)}")
        for g, s in zip(gradients, self.shapes):
            if g.shape != s or g.dtype != self.dtype or g.device.type != "cpu":
                raise RuntimeError("gradients must match the parameters' shapes, dtype and device")
        if is_distributed():
            raise RuntimeError("HostPowerSGD serves one process (world size 1)")
        self.step_counter += 1
        if self.step_counter <= self.config.start_compressing_after_num_steps:
            outs = [g.clone() for g in gradients]  # AllReduce at world size 1: copy, zero
            for g in gradients:
                g.zero_()
            return outs
        self._new_outputs()
        direct = self._pinned_in_place(gradients)
        if not direct:
            for i, g in enumerate(gradients):
                if self.is_compressed_mask[i]:
                    self._view(self.host_grads, i).copy_(g)
        # uncompressed: copy + zero on the host (world size 1 AllReduce)
        for i in self.unc:
            self._out_views[i].copy_(gradients[i])
            gradients[i].zero_()
        # pipeline: H2D (stream 0) -> codec (stream 1) -> D2H (stream 2), per device
        dres = self.residual_on_device
        for bn in self.bins:
            s_in, _, _ = self.streams[bn["dev"]]
            with torch.cuda.device(bn["dev"]), torch.cuda.stream(s_in):
                dst = bn["dstage"] if dres else bn["dflat"]
                dst.copy_(self.host_grads[bn["lo"]:bn["hi"]], non_blocking=True)
                bn["events"][0].record(s_in)
        for bn in self.bins:
            _, s_comp, _ = self.streams[bn["dev"]]
            with torch.cuda.device(bn["dev"]), torch.cuda.stream(s_comp):
                s_comp.wait_event(bn["events"][0])
                if dres:  # residual + fresh gradient (autograd's accumulation, on the device)
                    bn["dflat"].add_(bn["dstage"])
                bn["codec"].aggregate(bn["dgrads"])
                bn["events"][1].record(s_comp)
        for bn in self.bins:
            _, _, s_out = self.streams[bn["dev"]]
            with torch.cuda.device(bn["dev"]), torch.cuda.stream(s_out):
                s_out.wait_event(bn["events"][1])
                slab = bn["codec"]._slab.flat[:bn["hi"] - bn["lo"]]
                self.host_out[bn["lo"]:bn["hi"]].copy_(slab, non_blocking=True)
                if not dres:
                    self.host_grads[bn["lo"]:bn["hi"]].copy_(bn["dflat"], non_blocking=True)
        if dres:
            # the fresh gradients now live in the device residual: the compressed host ranges are
            # consumed (zeroed, as the reference leaves nothing of them in its inputs but the
            # residual), so a caller that skips zero_grad() cannot add them a second time. Each
            # bin is zeroed on the host as soon as its H2D copy has landed, under the GPU's codec
            # and D2H work.
            if not direct:
                for i, g in enumerate(gradients):
                    if self.is_compressed_mask[i]:
                        g.zero_()
            for bn in self.bins:
                bn["events"][0].synchronize()
                self.host_grads[bn["lo"]:bn["hi"]].zero_()
        for dev, (_, _, s_out) in self.streams.items():
            s_out.synchronize()
        if not direct and not dres:
            for i, g in enumerate(gradients):
                if self.is_compressed_mask[i]:
                    g.copy_(self._view(self.host_grads, i))
        return list(self._out_views)

    def residual(self) -> List[torch.Tensor]:
        """The compressed tensors' error-feedback residual (CPU copies; ``residual="device"``:
        from the GPU, synchronously). Uncompressed tensors have none (zero)."""
        out = [torch.zeros(s, dtype=self.dtype) for s in self.shapes]
        for bn in self.bins:
            host = bn["dflat"].cpu() if self.residual_on_device else self.host_grads[bn["lo"]:bn["hi"]]
            for i in bn["idx"]:
                out[i].copy_(self._view(host, i, base=bn["lo"]))
        return out
