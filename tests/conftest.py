import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libopk_hip.so)")


@pytest.fixture(scope="session")
def ctx():
    import torch
    from openpose_amd.api import Context
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    c = Context(0)
    yield c
    c.close()
