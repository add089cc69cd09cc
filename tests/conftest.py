import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def _gpu_test_drained(request):
    """Every GPU test ends with the device drained and its error state checked, so an
    asynchronous fault is reported by the test that caused it, not by a later one."""
    yield
    if request.node.get_closest_marker("gpu") is None or os.environ.get("RAGEN_AMD_NO_DRAIN") == "1":
        return
    import torch
    if torch.cuda.is_available():
        log = os.environ.get("RAGEN_AMD_PENDING_LOG")
        if log and not torch.cuda.current_stream().query():  # (diagnostic: work still queued at the test's end)
            with open(log, "a") as f:
                f.write(request.node.nodeid + "\n")
        torch.cuda.synchronize()
