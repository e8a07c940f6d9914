"""CPU checks of the collective-library override the GPU orchestration test relies on
(tests/test_gpu_rccl_stub.py): the stand-in library (tests/stubs/rccl_stub.hip) is built and
exports RCCL's entry points, and PSGD_RCCL_LIB_FORCE (with its second opt-in, PSGD_TESTING=1)
takes precedence over the RCCL already loaded in the process (torch's), read at every
psgd_comm_unique_id call; without the opt-in the override is ignored with a warning. Host-only
calls: no GPU is touched. The stub is test infrastructure built by `make test-stubs` (build()
runs it); these tests skip when it was not built."""
import ctypes
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(REPO, "tests", "stubs", "librccl_stub.so")
pytestmark = pytest.mark.skipif(not os.path.exists(STUB),
                                reason="tests/stubs/librccl_stub.so not built (make -C powersgd_amd/csrc test-stubs)")


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
        "os.environ['PSGD_TESTING'] = '1'\n"
        "c = _lib.comm_unique_id()\n"
        "print(a[:14] == b'psgd-rccl-stub', b[:14] == b'psgd-rccl-stub', c[:14] == b'psgd-rccl-stub')\n"
        % (REPO, STUB))
    env = {k: v for k, v in os.environ.items() if k not in ("PSGD_TESTING", "PSGD_RCCL_LIB_FORCE")}
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    # the override without its opt-in is ignored (and says so); with PSGD_TESTING=1 it wins
    assert p.stdout.strip().splitlines()[-1] == "False False True", p.stdout
    assert "PSGD_RCCL_LIB_FORCE" in p.stderr and "ignored" in p.stderr, p.stderr[-2000:]
    assert "collective library replaced" in p.stderr, p.stderr[-2000:]
