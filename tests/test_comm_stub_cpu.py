"""CPU checks of the collective-library override the GPU orchestration test relies on
(tests/test_gpu_rccl_stub.py): the stand-in library (tests/stubs/rccl_stub.hip) is built and
exports RCCL's entry points, and PSGD_RCCL_LIB_FORCE takes precedence over the RCCL already
loaded in the process (torch's), read at every psgd_comm_unique_id call. Host-only calls: no
GPU is touched."""
import ctypes
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(REPO, "tests", "stubs", "librccl_stub.so")


def test_stub_library_exports_rccl_entry_points():
    lib = ctypes.CDLL(STUB)
    for name in ("ncclGetUniqueId", "ncclCommInitRank", "ncclCommDestroy", "ncclAllReduce", "ncclGroupStart",
                 "ncclGroupEnd", "ncclGetErrorString", "psgd_stub_calls"):
        assert hasattr(lib, name), name
    uid = (ctypes.c_uint8 * 128)()
    assert lib.ncclGetUniqueId(uid) == 0
    assert bytes(uid)[:14] == b"psgd-rccl-stub"


def test_forced_library_wins_over_the_process_rccl():
    """In a fresh process that has imported torch (whose RCCL is then in the process), the
    communicator id comes from the forced stand-in, and from the real RCCL without the override."""
    code = (
        "import os, sys, torch; sys.path.insert(0, %r)\n"
        "from powersgd_amd import _lib\n"
        "a = _lib.comm_unique_id()\n"
        "os.environ['PSGD_RCCL_LIB_FORCE'] = %r\n"
        "b = _lib.comm_unique_id()\n"
        "print(a[:14] == b'psgd-rccl-stub', b[:14] == b'psgd-rccl-stub')\n" % (REPO, STUB))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    assert p.stdout.strip().splitlines()[-1] == "False True", p.stdout
