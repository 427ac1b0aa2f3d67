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


_REPORTED = []


def pytest_runtest_logreport(report):
    """Collect the measured quantities tests publish with record_property("report_...", value)
    (e.g. the full-strength keypoint parity), so that they are printed at the end of the run."""
    if report.when == "call":
        for k, v in report.user_properties:
            if k.startswith("report_"):
                _REPORTED.append((report.nodeid, k[len("report_"):], v))


def pytest_terminal_summary(terminalreporter):
    if _REPORTED:
        terminalreporter.section("measured (record_property report_*)")
        for nodeid, k, v in _REPORTED:
            terminalreporter.write_line("%s: %s = %s" % (nodeid.split("::")[-1], k, v))
