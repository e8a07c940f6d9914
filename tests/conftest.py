import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: full-size (BASELINE config) cases")


@pytest.fixture(autouse=True)
def _restore_default_dtype():
    # the reference's own test flips the global default dtype (tests/powersgd_test.py:38);
    # keep that from leaking between our tests
    import torch

    prev = torch.get_default_dtype()
    yield
    torch.set_default_dtype(prev)
