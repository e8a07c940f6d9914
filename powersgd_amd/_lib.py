"""ctypes binding of libpsgd.so (the C ABI in include/psgd.h).

The library is built in-tree (powersgd_amd/_lib/libpsgd.so, see powersgd_amd/csrc/Makefile).
There is no fallback: if the library is missing, every compute entry point raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
# PSGD_LIB_PATH: an alternative in-tree build (tuning variants); default the standard one
LIB_PATH = os.environ.get("PSGD_LIB_PATH") or os.path.join(_HERE, "_lib", "libpsgd.so")

PSGD_F32, PSGD_BF16, PSGD_F64 = 0, 1, 2
_STATUS_NAMES = {1: "INDEX", 2: "VALUE", 3: "DTYPE", 4: "LAYOUT", 5: "DEVICE", 6: "STATE"}

_i32, _i64, _dbl, _vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p
_P_i64, _P_i32, _P_dbl = ctypes.POINTER(_i64), ctypes.POINTER(_i32), ctypes.POINTER(_dbl)

_SIGNATURES = {
    "psgd_version": ([], _i32),
    "psgd_last_error": ([], ctypes.c_char_p),
    "psgd_should_compress": ([_P_i64, _i32, _i32, _i32, _dbl, _P_i32], _i32),
    "psgd_plan_create": ([_P_i64, _P_i32, _i32, _i32, _i32, _i32, ctypes.POINTER(_vp)], _i32),
    "psgd_plan_destroy": ([_vp], _i32),
    "psgd_plan_num_groups": ([_vp, _P_i32], _i32),
    "psgd_plan_group": ([_vp, _i32, _P_i64, _P_i64, _P_i32, _P_i32], _i32),
    "psgd_plan_factor_numel": ([_vp, _P_i64, _P_i64], _i32),
    "psgd_plan_output_offset": ([_vp, _i32, _P_i64], _i32),
    "psgd_plan_output_numel": ([_vp, _P_i64], _i32),
    "psgd_plan_workspace_bytes": ([_vp, _P_i64], _i32),
    "psgd_plan_compression_rate": ([_vp, _P_dbl, _P_dbl, _P_dbl], _i32),
    "psgd_plan_bind": ([_vp, _i32, _vp, _vp, _vp], _i32),
    "psgd_out_factor": ([_vp, _i64, _i32, _P_i32], _i32),
    "psgd_compress": ([_vp, _vp, _i64, _i32, _vp], _i32),
    "psgd_decompress": ([_vp, _vp, _vp, _i64, _i32, _vp], _i32),
    "psgd_aggregate": ([_vp, _vp, _vp, _i64, _vp], _i32),
    "psgd_plan_fused_final": ([_vp, _i64, _i32, _P_i32], _i32),
    "psgd_plan_odd_even": ([_vp, _i64, _i32, _P_i32], _i32),
    "psgd_plan_set_timing": ([_vp, _i32], _i32),
    "psgd_plan_timing_read": ([_vp, _P_dbl, _P_i32], _i32),
    "psgd_flat_create": ([_P_i64, _i32, _i32, ctypes.POINTER(_vp)], _i32),
    "psgd_flat_destroy": ([_vp], _i32),
    "psgd_flat_workspace_bytes": ([_vp, _P_i64], _i32),
    "psgd_flat_bind": ([_vp, _i32, _vp], _i32),
    "psgd_flat_pack": ([_vp, _vp, _vp, _i32, _vp], _i32),
    "psgd_aggregate_flat": ([_vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp], _i32),
    "psgd_product": ([_vp, _vp, _i32, _vp, _vp, _i32, _vp, _vp, _vp], _i32),
    "psgd_orthogonalize": ([_vp, _i32, _vp, _i32, _vp], _i32),
    "psgd_reconstruct": ([_vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, ctypes.c_float, _vp], _i32),
    "psgd_plan_set_buckets": ([_vp, _i32, _P_i32], _i32),
    "psgd_plan_bucket_range": ([_vp, _i32, _P_i64, _P_i64, _P_i64, _P_i64], _i32),
    "psgd_compress_bucket": ([_vp, _vp, _i64, _i32, _i32, _vp], _i32),
    "psgd_decompress_bucket": ([_vp, _vp, _vp, _i64, _i32, _i32, _vp], _i32),
    "psgd_comm_id_bytes": ([_P_i64], _i32),
    "psgd_comm_unique_id": ([_vp], _i32),
    "psgd_comm_init": ([_i32, _i32, _vp, _i32, ctypes.POINTER(_vp)], _i32),
    "psgd_comm_destroy": ([_vp], _i32),
    "psgd_aggregate_comm": ([_vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp], _i32),
    "psgd_ipc_handle_bytes": ([_P_i64], _i32),
    "psgd_ipc_create": ([_vp, _i64, _vp], _i32),
    "psgd_ipc_open": ([_vp, _i32, _i32, _vp], _i32),
    "psgd_aggregate_ipc": ([_vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp], _i32),
    "psgd_ipc_status": ([_vp, _P_i32], _i32),
    "psgd_ipc_close": ([_vp], _i32),
    "psgd_ipc_debug": ([_vp, _i32, _vp], _i32),
    "psgd_runs_create": ([_P_i64, _P_i32, _P_i64, _P_i64, _i32, _i32, _i32, ctypes.POINTER(_vp)], _i32),
    "psgd_runs_destroy": ([_vp], _i32),
    "psgd_runs_workspace_bytes": ([_vp, _P_i64], _i32),
    "psgd_runs_bind": ([_vp, _i32, _vp], _i32),
    "psgd_runs_add": ([_vp, _vp, _vp, _vp], _i32),
    "psgd_runs_gather": ([_vp, _vp, _vp, _vp], _i32),
}

EXPORTED_SYMBOLS = tuple(_SIGNATURES)


class _IpcInfo(ctypes.Structure):  # psgd_ipc_info (include/psgd.h)
    _fields_ = [("arena_allocs", _i64), ("arena_opens", _i64), ("arena_reuses", _i64), ("arena_frees", _i64),
                ("own_va", ctypes.c_uint64), ("peer_va", ctypes.c_uint64), ("own_nonce", ctypes.c_uint32),
                ("peer_nonce_seen", ctypes.c_uint32)]

_lib = None


class LibraryMissing(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    """Load libpsgd.so once; raise loudly when it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise LibraryMissing(
                f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "or `make -C powersgd_amd/csrc`. powersgd_amd has no CPU fallback."
            )
        handle = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in _SIGNATURES.items():
            fn = getattr(handle, name)
            fn.argtypes = args
            fn.restype = res
        _lib = handle
    return _lib


def check(status: int) -> None:
    if status == 0:
        return
    msg = lib().psgd_last_error().decode(errors="replace")
    name = _STATUS_NAMES.get(status, str(status))
    if status == 1:
        raise IndexError(msg)
    if status == 2:
        raise ValueError(msg)
    raise RuntimeError(f"psgd error {name}: {msg}")


def shape_arrays(shapes: Sequence[Sequence[int]]):
    flat: List[int] = [int(d) for s in shapes for d in s]
    dims = (_i64 * max(1, len(flat)))(*flat)
    ndims = (_i32 * max(1, len(shapes)))(*[len(s) for s in shapes])
    return dims, ndims


def ptr_array(ptrs: Sequence[int]):
    return (_vp * max(1, len(ptrs)))(*ptrs)


class Plan:
    """Owns a psgd_plan handle (host layout only; device memory is bound by the caller)."""

    def __init__(self, shapes: Sequence[Sequence[int]], rank: int, iters: int, dtype_code: int):
        L = lib()
        dims, ndims = shape_arrays(shapes)
        h = _vp()
        check(L.psgd_plan_create(dims, ndims, len(shapes), rank, iters, dtype_code, ctypes.byref(h)))
        self._h = h
        self.num_tensors = len(shapes)
        self.iters = iters

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib is not None:
            _lib.psgd_plan_destroy(h)
            self._h = None

    # --- layout queries
    def groups(self):
        L, n_ = lib(), _i32()
        check(L.psgd_plan_num_groups(self._h, ctypes.byref(n_)))
        out = []
        for g in range(n_.value):
            n, m, r, c = _i64(), _i64(), _i32(), _i32()
            check(L.psgd_plan_group(self._h, g, ctypes.byref(n), ctypes.byref(m), ctypes.byref(r), ctypes.byref(c)))
            out.append((n.value, m.value, r.value, c.value))
        return out

    def factor_numel(self):
        p, q = _i64(), _i64()
        check(lib().psgd_plan_factor_numel(self._h, ctypes.byref(p), ctypes.byref(q)))
        return p.value, q.value

    def output_numel(self) -> int:
        n = _i64()
        check(lib().psgd_plan_output_numel(self._h, ctypes.byref(n)))
        return n.value

    def output_offsets(self) -> List[int]:
        out, o = [], _i64()
        for i in range(self.num_tensors):
            check(lib().psgd_plan_output_offset(self._h, i, ctypes.byref(o)))
            out.append(o.value)
        return out

    def workspace_bytes(self) -> int:
        b = _i64()
        check(lib().psgd_plan_workspace_bytes(self._h, ctypes.byref(b)))
        return b.value

    def compression_rate(self):
        r, u, c = _dbl(), _dbl(), _dbl()
        check(lib().psgd_plan_compression_rate(self._h, ctypes.byref(r), ctypes.byref(u), ctypes.byref(c)))
        return r.value, u.value, c.value

    # --- device
    def bind(self, device: int, p_ptr: int, q_ptr: int, ws_ptr: int) -> None:
        check(lib().psgd_plan_bind(self._h, device, p_ptr, q_ptr, ws_ptr))

    def out_factor(self, step: int, it: int) -> int:
        w = _i32()
        check(lib().psgd_out_factor(self._h, step, it, ctypes.byref(w)))
        return w.value

    def compress(self, grads, step: int, it: int, stream: int) -> None:
        check(lib().psgd_compress(self._h, grads, step, it, stream))

    def decompress(self, grads, out_ptr: int, step: int, world: int, stream: int) -> None:
        check(lib().psgd_decompress(self._h, grads, out_ptr, step, world, stream))

    def aggregate(self, grads, out_ptr: int, step: int, stream: int) -> None:
        check(lib().psgd_aggregate(self._h, grads, out_ptr, step, stream))

    def aggregate_flat(self, grads, out_ptr: int, step: int, flat: "FlatPlan", unc, flat_out: int,
                       stream: int) -> None:
        check(lib().psgd_aggregate_flat(self._h, grads, out_ptr, step, flat._h, unc, flat_out, stream))

    # --- buckets of shape groups (W > 1 comm/compute overlap)
    def set_buckets(self, group_end: Sequence[int]) -> None:
        arr = (_i32 * max(1, len(group_end)))(*group_end)
        check(lib().psgd_plan_set_buckets(self._h, len(group_end), arr))

    def bucket_range(self, b: int):
        po, pl, qo, ql = _i64(), _i64(), _i64(), _i64()
        check(lib().psgd_plan_bucket_range(self._h, b, ctypes.byref(po), ctypes.byref(pl), ctypes.byref(qo),
                                           ctypes.byref(ql)))
        return po.value, pl.value, qo.value, ql.value

    def aggregate_comm(self, grads, out_ptr: int, step: int, flat, unc, flat_out: int, comm: "Comm",
                       stream: int) -> None:
        check(lib().psgd_aggregate_comm(self._h, grads, out_ptr, step, flat._h if flat else None, unc, flat_out,
                                        comm._h, stream))

    def compress_bucket(self, grads, step: int, it: int, bucket: int, stream: int) -> None:
        check(lib().psgd_compress_bucket(self._h, grads, step, it, bucket, stream))

    def decompress_bucket(self, grads, out_ptr: int, step: int, world: int, bucket: int, stream: int) -> None:
        check(lib().psgd_decompress_bucket(self._h, grads, out_ptr, step, world, bucket, stream))

    # --- one-shot all-reduce over IPC exchange buffers, device-side flags (W > 1, one node)
    def ipc_create(self, flat_numel: int = 0) -> bytes:
        n = _i64()
        check(lib().psgd_ipc_handle_bytes(ctypes.byref(n)))
        buf = (ctypes.c_uint8 * n.value)()
        check(lib().psgd_ipc_create(self._h, flat_numel, buf))
        return bytes(buf)

    def ipc_open(self, world: int, rank: int, handles: Sequence[bytes]) -> None:
        blob = b"".join(handles)
        arr = (ctypes.c_uint8 * len(blob)).from_buffer_copy(blob)
        check(lib().psgd_ipc_open(self._h, world, rank, arr))

    def aggregate_ipc(self, grads, out_ptr: int, step: int, flat, unc, flat_out: int, stream: int) -> None:
        check(lib().psgd_aggregate_ipc(self._h, grads, out_ptr, step, flat._h if flat else None, unc, flat_out,
                                       stream))

    def ipc_status(self) -> bool:
        """True if a device-side wait timed out since the exchange was opened (synchronous; sticky
        until ipc_close: every later aggregate_ipc raises)."""
        v = _i32()
        check(lib().psgd_ipc_status(self._h, ctypes.byref(v)))
        return bool(v.value)

    def ipc_close(self) -> None:
        check(lib().psgd_ipc_close(self._h))

    def ipc_debug(self, peer: int = 0) -> dict:
        """psgd_ipc_debug: the process's exchange-arena counters, this session's region address
        and nonce, and peer `peer`'s mapped region address and the nonce read through it."""
        info = _IpcInfo()
        check(lib().psgd_ipc_debug(self._h, peer, ctypes.byref(info)))
        return {f: int(getattr(info, f)) for f, _ in _IpcInfo._fields_}

    def fused_final(self, step: int, aggregate: bool = True) -> int:
        """Nonzero when the last iteration of ``step`` runs fused with the final pass: 2 in the
        projection form, 1 in the K-term form (``aggregate``: in ``psgd_aggregate``, the
        world-size-1 path; else the building blocks)."""
        f = _i32()
        check(lib().psgd_plan_fused_final(self._h, step, 1 if aggregate else 0, ctypes.byref(f)))
        return int(f.value)

    def odd_even(self, step: int, it: int) -> bool:
        """True when odd iteration ``it`` of ``step`` runs fused with the next (even) iteration's
        product in one gradient pass (psgd_aggregate: rank 1, world size 1, I >= 3)."""
        f = _i32()
        check(lib().psgd_plan_odd_even(self._h, step, it, ctypes.byref(f)))
        return bool(f.value)

    # --- building blocks (paper-code reducer variants, powersgd_amd/reducers.py)
    def product(self, grads, odd: bool, x_ptr: int, y_ptr: int, terms=(), stream: int = 0) -> None:
        tp = ptr_array([t[0] for t in terms]) if terms else None
        tq = ptr_array([t[1] for t in terms]) if terms else None
        check(lib().psgd_product(self._h, grads, 1 if odd else 0, x_ptr, y_ptr, len(terms), tp, tq, stream))

    def orthogonalize(self, which_p: bool, buf_ptr: int, mode: int, stream: int) -> None:
        check(lib().psgd_orthogonalize(self._h, 1 if which_p else 0, buf_ptr, mode, stream))

    def reconstruct(self, grads, resid_out, out, terms, avg_terms, alpha: float, stream: int) -> None:
        tp = ptr_array([t[0] for t in terms])
        tq = ptr_array([t[1] for t in terms])
        ap = ptr_array([t[0] for t in avg_terms])
        aq = ptr_array([t[1] for t in avg_terms])
        check(lib().psgd_reconstruct(self._h, grads, resid_out, out, len(terms), tp, tq, ap, aq, alpha, stream))

    def set_timing(self, enable: bool) -> None:
        check(lib().psgd_plan_set_timing(self._h, 1 if enable else 0))

    def timing_read(self):
        """(summed k_apply milliseconds, launches) since timing was enabled / last read."""
        ms, n = _dbl(), _i32()
        check(lib().psgd_plan_timing_read(self._h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value


class FlatPlan:
    def __init__(self, numels: Sequence[int], dtype_code: int):
        L = lib()
        arr = (_i64 * max(1, len(numels)))(*numels)
        h = _vp()
        check(L.psgd_flat_create(arr, len(numels), dtype_code, ctypes.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib is not None:
            _lib.psgd_flat_destroy(h)
            self._h = None

    def workspace_bytes(self) -> int:
        b = _i64()
        check(lib().psgd_flat_workspace_bytes(self._h, ctypes.byref(b)))
        return b.value

    def bind(self, device: int, ws_ptr: int) -> None:
        check(lib().psgd_flat_bind(self._h, device, ws_ptr))

    def pack(self, tensors, flat_ptr: int, world: int, stream: int) -> None:
        check(lib().psgd_flat_pack(self._h, tensors, flat_ptr, world, stream))


class Runs:
    """Owns a psgd_runs: a DDP bucket's flat buffer <-> per-parameter tensors (run table, 64-bit
    offsets). ``add``: tensors += bucket (error-feedback add); ``gather``: bucket = tensors."""

    def __init__(self, bucket_off: Sequence[int], tensor: Sequence[int], tensor_off: Sequence[int],
                 length: Sequence[int], ntensors: int, dtype_code: int):
        n = len(length)
        h = _vp()
        check(lib().psgd_runs_create((_i64 * max(1, n))(*bucket_off), (_i32 * max(1, n))(*tensor),
                                     (_i64 * max(1, n))(*tensor_off), (_i64 * max(1, n))(*length), n, ntensors,
                                     dtype_code, ctypes.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib is not None:
            _lib.psgd_runs_destroy(h)
            self._h = None

    def workspace_bytes(self) -> int:
        b = _i64()
        check(lib().psgd_runs_workspace_bytes(self._h, ctypes.byref(b)))
        return b.value

    def bind(self, device: int, ws_ptr: int) -> None:
        check(lib().psgd_runs_bind(self._h, device, ws_ptr))

    def add(self, bucket_ptr: int, tensors, stream: int) -> None:
        check(lib().psgd_runs_add(self._h, bucket_ptr, tensors, stream))

    def gather(self, bucket_ptr: int, tensors, stream: int) -> None:
        check(lib().psgd_runs_gather(self._h, bucket_ptr, tensors, stream))


def comm_unique_id() -> bytes:
    """RCCL communicator id (rank 0); the caller broadcasts it to every rank."""
    n = _i64()
    check(lib().psgd_comm_id_bytes(ctypes.byref(n)))
    buf = (ctypes.c_uint8 * n.value)()
    check(lib().psgd_comm_unique_id(buf))
    return bytes(buf)


class Comm:
    """Owns a psgd_comm: an RCCL communicator the library drives on the codec's stream."""

    def __init__(self, world: int, rank: int, uid: bytes, device: int):
        arr = (ctypes.c_uint8 * len(uid)).from_buffer_copy(uid)
        h = _vp()
        check(lib().psgd_comm_init(world, rank, arr, device, ctypes.byref(h)))
        self._h = h
        self.world = world

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib is not None:
            _lib.psgd_comm_destroy(h)
            self._h = None


def should_compress(shape: Sequence[int], rank: int, iters: int, min_rate: float) -> bool:
    dims, _ = shape_arrays([shape])
    out = _i32()
    check(lib().psgd_should_compress(dims, len(shape), rank, iters, float(min_rate), ctypes.byref(out)))
    return bool(out.value)
