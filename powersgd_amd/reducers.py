"""The paper code's PowerSGD reducers on the MI355X codec.

``RankKReducer`` (reference paper-code/gradient_reducers.py:665-788) and
``HalfRankKReducer`` (:794-936) with the paper's interface:
``reduce(grad_in, grad_out, memory_out) -> bits communicated``; ``grad_in`` is read,
``grad_out`` receives the averaged approximation and ``memory_out`` the error-feedback
memory (the paper's training loop passes ``send = grad + memory``, train.py:177-186).

Every matrix step runs on the codec's HIP kernels through the C ABI building blocks
(include/psgd.h: ``psgd_product``, ``psgd_orthogonalize`` mode 1 = the paper's Gram-Schmidt
with the eps added to the norm, ``psgd_reconstruct`` writing memory and output straight into
the caller's tensors). Factor buffers follow the codec's shape-grouped layout instead of the
paper's tensor-order ``p_memory`` / ``q_memory``; the all-reduce is a SUM over the whole
buffer either way, so only the element order differs. Tensors with one dimension are
averaged uncompressed, as in the paper. The query draws are the paper's (``torch.manual_seed
(rng.randint(1e9))`` then ``torch.randn`` on the device); ``random_fn`` overrides them
(tests inject the draws the paper code made on CPU).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Callable, Dict, List, Optional

import numpy as np
import torch

from . import _lib
from .powersgd import _dtype_code, _require_device, _stream
from .utils import is_distributed


def _bits(t: torch.Tensor) -> int:
    return 8 * t.nelement() * t.element_size()  # paper n_bits (:1123-1124)


class _Codec:
    """Plan + fp32 factor buffers (codec layout) for the paper's high-rank tensors."""

    def __init__(self, tensors: List[torch.Tensor], rank: int):
        t0 = tensors[0]
        self.device = t0.device
        self.dev_index = _require_device(t0.device)
        self.shapes = [t.shape for t in tensors]
        # the codec's matrix view is [shape[0], numel/shape[0]] (as the paper's view(n, -1))
        self.plan = _lib.Plan([tuple(s) for s in self.shapes], rank, 2, _dtype_code(t0.dtype))
        pn, qn = self.plan.factor_numel()
        self.P = torch.zeros(pn, dtype=torch.float32, device=self.device)
        self.Q = torch.zeros(qn, dtype=torch.float32, device=self.device)
        self.ws = torch.empty(self.plan.workspace_bytes(), dtype=torch.uint8, device=self.device)
        self.plan.bind(self.dev_index, self.P.data_ptr(), self.Q.data_ptr(), self.ws.data_ptr())
        # per-tensor views of P / Q in the codec layout (shape groups, first appearance)
        groups: "OrderedDict[tuple, List[int]]" = OrderedDict()
        for i, s in enumerate(self.shapes):
            n = s[0]
            groups.setdefault((n, s.numel() // n), []).append(i)
        self.pv: Dict[int, torch.Tensor] = {}
        self.qv: Dict[int, torch.Tensor] = {}
        po = qo = 0
        for (n, m), idx in groups.items():
            r = min(rank, n, m)
            for i in idx:
                self.pv[i] = self.P[po:po + n * r].view(n, r)
                self.qv[i] = self.Q[qo:qo + m * r].view(m, r)
                po += n * r
                qo += m * r

    def ptrs(self, tensors: List[torch.Tensor]):
        for t in tensors:
            if not t.is_contiguous():
                raise RuntimeError("view size is not compatible with input tensor's size and stride")
        return _lib.ptr_array([t.data_ptr() for t in tensors])


class _PaperReducer:
    def __init__(self, random_seed: int, device, timer=None, rank: int = 1,
                 random_fn: Optional[Callable] = None):
        self.rng = np.random.RandomState(random_seed)  # paper Reducer.__init__ (:16-29)
        self.device = torch.device(device)
        self.timer = timer
        self.rank = rank
        self.random_fn = random_fn
        self.n_workers = torch.distributed.get_world_size() if is_distributed() else 1
        self._codec: Optional[_Codec] = None

    def _draw(self, vector: torch.Tensor) -> None:
        """set_random's draw (:674-676 / :807-809)."""
        if self.random_fn is not None:
            vector.copy_(self.random_fn(tuple(vector.shape)))
            return
        torch.manual_seed(self.rng.randint(1_000_000_000))
        vector.copy_(torch.randn(*vector.shape, device=self.device))

    def _split(self, grad_in, grad_out, memory_out):
        high = [i for i, t in enumerate(grad_in) if t.ndimension() > 1]
        rank1 = [i for i, t in enumerate(grad_in) if t.ndimension() <= 1]
        return high, rank1

    def _all_reduce(self, t: torch.Tensor, async_op: bool = False):
        if is_distributed() and torch.distributed.get_world_size() > 1:  # paper all_reduce (:1183-1185)
            return torch.distributed.all_reduce(t, async_op=async_op)
        return None


class RankKReducer(_PaperReducer):
    """paper-code/gradient_reducers.py:665-788 (n_power_iterations = 0)."""

    def __init__(self, random_seed, device, timer=None, n_power_iterations=0, reuse_query=False, rank=1,
                 random_fn: Optional[Callable] = None):
        super().__init__(random_seed, device, timer, rank, random_fn)
        assert n_power_iterations == 0
        self.reuse_query = reuse_query

    def reduce(self, grad_in, grad_out, memory_out) -> int:
        bits = 0
        high, rank1 = self._split(grad_in, grad_out, memory_out)
        uninit = self._codec is None
        if self._codec is None:
            self._codec = _Codec([grad_in[i] for i in high], self.rank)
        c = self._codec
        s = _stream(c.device)
        g = c.ptrs([grad_in[i] for i in high])
        if not (self.reuse_query and not uninit):  # :735-745
            for k in range(len(high)):
                self._draw(c.qv[k])
        c.plan.product(g, True, c.Q.data_ptr(), c.P.data_ptr(), (), s)  # p = M q (:747-750)
        self._all_reduce(c.P)  # :752-754
        bits += _bits(c.P)
        buf = torch.cat([grad_in[i].view(-1) for i in rank1]) if rank1 else None  # :756-761
        handle = self._all_reduce(buf, async_op=True) if buf is not None else None
        if buf is not None:
            bits += _bits(buf)
        c.plan.orthogonalize(True, c.P.data_ptr(), 1, s)  # :763-765
        c.plan.product(g, False, c.P.data_ptr(), c.Q.data_ptr(), (), s)  # q = M^T p (:767-770)
        self._all_reduce(c.Q)  # :772-775
        bits += _bits(c.Q)
        if self.n_workers > 1:
            c.Q.div_(self.n_workers)
        term = (c.P.data_ptr(), c.Q.data_ptr())
        c.plan.reconstruct(g, c.ptrs([memory_out[i] for i in high]), c.ptrs([grad_out[i] for i in high]),
                           [term], [term], 1.0, s)  # out = p q^T, mem = M - out (:777-781)
        if buf is not None:  # :783-786
            if handle is not None:
                handle.wait()
            buf /= self.n_workers
            o = 0
            for i in rank1:
                grad_out[i].copy_(buf[o:o + grad_out[i].numel()].view(grad_out[i].shape))
                o += grad_out[i].numel()
        return bits


class HalfRankKReducer(_PaperReducer):
    """paper-code/gradient_reducers.py:794-936 (one product per step, alternating)."""

    def __init__(self, random_seed, device, timer=None, rank=1, random_fn: Optional[Callable] = None):
        super().__init__(random_seed, device, timer, rank, random_fn)
        self.next_operation = "p"

    def reduce(self, grad_in, grad_out, memory_out) -> int:
        bits = 0
        high, rank1 = self._split(grad_in, grad_out, memory_out)
        buf = torch.cat([grad_in[i].view(-1) for i in rank1]) if rank1 else None  # :833-839
        handle = self._all_reduce(buf, async_op=True) if buf is not None else None
        if buf is not None:
            bits += _bits(buf)
        uninit = self._codec is None
        if self._codec is None:
            self._codec = _Codec([grad_in[i] for i in high], self.rank)
        c = self._codec
        s = _stream(c.device)
        g = c.ptrs([grad_in[i] for i in high])
        mem = c.ptrs([memory_out[i] for i in high])
        out = c.ptrs([grad_out[i] for i in high])
        W = self.n_workers
        if self.next_operation == "p":  # :875-902
            self.next_operation = "q"
            if uninit:
                for k in range(len(high)):
                    self._draw(c.qv[k])
            c.plan.orthogonalize(False, c.Q.data_ptr(), 1, s)  # set_random's / the step's orthogonalize
            c.plan.product(g, True, c.Q.data_ptr(), c.P.data_ptr(), (), s)
            local = c.P.clone() if W > 1 else c.P
            self._all_reduce(c.P)
            bits += _bits(c.P)
            if W > 1:
                c.P.div_(W)
            q = c.Q.data_ptr()
            c.plan.reconstruct(g, mem, out, [(local.data_ptr(), q)], [(c.P.data_ptr(), q)], 1.0, s)
        else:  # :904-927
            self.next_operation = "p"
            c.plan.orthogonalize(True, c.P.data_ptr(), 1, s)
            c.plan.product(g, False, c.P.data_ptr(), c.Q.data_ptr(), (), s)
            local = c.Q.clone() if W > 1 else c.Q
            self._all_reduce(c.Q)
            bits += _bits(c.Q)
            if W > 1:
                c.Q.div_(W)
            p = c.P.data_ptr()
            c.plan.reconstruct(g, mem, out, [(p, local.data_ptr())], [(p, c.Q.data_ptr())], 1.0, s)
        if buf is not None:  # :929-936
            if handle is not None:
                handle.wait()
            buf /= W
            o = 0
            for i in rank1:
                grad_out[i].copy_(buf[o:o + grad_out[i].numel()].view(grad_out[i].shape))
                o += grad_out[i].numel()
        return bits
