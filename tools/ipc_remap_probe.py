"""Does HIP hand back a stale IPC mapping after a free -> malloc -> re-export cycle?

The round-5 exchange (one hipMalloc per session, hipFree at plan destruction, peers
hipIpcOpenMemHandle'd per session) failed once with wrong sums exactly when a second same-size
session followed a closed one in the same processes (gpurun_out/r05a-new.log). This probe
replays that allocation pattern with the raw HIP runtime, two processes on one GPU:

  A: X = hipMalloc(n); fill X with 1; export h1          B: open h1 -> va1; read; close
  A: hipFree(X); X' = hipMalloc(n); fill X' with 2; export h2
                                                          B: open h2 -> va2; read
and reports, per round: A's addresses (X == X'?), whether h1 == h2 byte for byte, B's mapped
addresses, and what B reads through the second mapping (2 = correct; 1 = the freed buffer's
bytes, i.e. a stale mapping). Several rounds and sizes (the r05 exchange buffers were 1-8 MB).

usage (GPU box): python tools/ipc_remap_probe.py [rounds]
"""
import ctypes
import json
import os
import sys
import tempfile

HIP = "/opt/rocm/lib/libamdhip64.so"


class IpcHandle(ctypes.Structure):  # hipIpcMemHandle_t, passed BY VALUE to hipIpcOpenMemHandle
    _fields_ = [("reserved", ctypes.c_char * 64)]


def _hip():
    # the HIP runtime torch already loaded (its bundled ROCm); /opt/rocm's does not load beside it
    import torch  # noqa: F401

    lib = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    h = ctypes.CDLL(lib if os.path.exists(lib) else HIP)
    h.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    h.hipFree.argtypes = [ctypes.c_void_p]
    h.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
    h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    h.hipIpcGetMemHandle.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    h.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), IpcHandle, ctypes.c_uint]
    h.hipIpcCloseMemHandle.argtypes = [ctypes.c_void_p]
    h.hipDeviceSynchronize.argtypes = []
    h.hipSetDevice.argtypes = [ctypes.c_int]
    return h


def _ok(e, what):
    if e != 0:
        raise RuntimeError(f"{what}: hip error {e}")


def _exporter(h, n, value):
    p = ctypes.c_void_p()
    _ok(h.hipMalloc(ctypes.byref(p), n), "hipMalloc")
    _ok(h.hipMemset(p, value, n), "hipMemset")
    _ok(h.hipDeviceSynchronize(), "sync")
    hb = IpcHandle()
    _ok(h.hipIpcGetMemHandle(ctypes.byref(hb), p), "hipIpcGetMemHandle")
    return p, bytes(ctypes.string_at(ctypes.addressof(hb), 64))


def _read(h, va, n):
    buf = (ctypes.c_uint8 * 16)()
    _ok(h.hipMemcpy(buf, ctypes.c_void_p(va + n // 2), 16, 2), "hipMemcpy D2H")  # middle of the buffer
    return sorted(set(buf))


def worker(rank, initfile, rounds, sizes, out, keep_open=False):
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"file://{initfile}", rank=rank, world_size=2)
    h = _hip()
    _ok(h.hipSetDevice(0), "hipSetDevice")
    recs = []
    for n in sizes:
        for r in range(rounds):
            msg = [None]
            if rank == 0:
                x1, h1 = _exporter(h, n, 1)
                msg = [(x1.value, h1)]
            dist.broadcast_object_list(msg, src=0)
            if rank == 1:
                va1 = ctypes.c_void_p()
                _ok(h.hipIpcOpenMemHandle(ctypes.byref(va1), IpcHandle.from_buffer_copy(msg[0][1]), 1),
                    "open h1")
                seen1 = _read(h, va1.value, n)
                if not keep_open:
                    _ok(h.hipIpcCloseMemHandle(va1), "close h1")
            dist.barrier()
            if rank == 0:
                _ok(h.hipFree(x1), "hipFree")
                x2, h2 = _exporter(h, n, 2)
                msg2 = [(x2.value, h2, x1.value, h1)]
            else:
                msg2 = [None]
            dist.broadcast_object_list(msg2, src=0)
            if rank == 1:
                a2, hh2, a1, hh1 = msg2[0]
                va2 = ctypes.c_void_p()
                e = h.hipIpcOpenMemHandle(ctypes.byref(va2), IpcHandle.from_buffer_copy(hh2), 1)
                seen2 = _read(h, va2.value, n) if e == 0 else None
                if e == 0:
                    _ok(h.hipIpcCloseMemHandle(va2), "close h2")
                if keep_open and va2.value != va1.value:
                    _ok(h.hipIpcCloseMemHandle(va1), "close h1")
                recs.append({"keep_first_mapping_open": keep_open, "bytes": n, "round": r, "exporter_same_va": a1 == a2, "handles_equal": hh1 == hh2,
                             "handle_diff_bytes": [i for i in range(64) if hh1[i] != hh2[i]],
                             "importer_va1": hex(va1.value), "importer_va2": hex(va2.value or 0),
                             "importer_same_va": va1.value == va2.value, "open2_error": e,
                             "seen_first": seen1, "seen_second": seen2,
                             "stale": seen2 is not None and seen2 != [2]})
            dist.barrier()
            if rank == 0:
                _ok(h.hipFree(x2), "hipFree")
    if rank == 1:
        with open(out, "w") as f:
            for rec in recs:
                f.write(json.dumps(rec) + "\n")
    dist.barrier()
    dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp

    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    sizes = [1 << 20, 3 << 20, 8 << 20, 64 << 20]
    # scenario 1: the importer closes its mapping before the owner frees (the documented
    # teardown); scenario 2: the importer still holds the first mapping when the owner frees and
    # re-allocates (a teardown out of order, or a second mapping of the same buffer left open)
    for keep_open in (False, True):
        with tempfile.TemporaryDirectory() as td:
            out = os.path.join(td, "recs.jsonl")
            mp.spawn(worker, args=(os.path.join(td, "init"), rounds, sizes, out, keep_open), nprocs=2, join=True)
            recs = [json.loads(x) for x in open(out)]
        for rec in recs:
            print(json.dumps(rec))
        print(json.dumps({"summary": {"keep_first_mapping_open": keep_open, "rounds": len(recs),
                                      "stale": sum(r["stale"] for r in recs),
                                      "exporter_same_va": sum(r["exporter_same_va"] for r in recs),
                                      "handles_equal": sum(r["handles_equal"] for r in recs),
                                      "importer_same_va": sum(r["importer_same_va"] for r in recs)}}))


if __name__ == "__main__":
    main()
