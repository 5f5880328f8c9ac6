import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libsm_hip.so on the GPU)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.load()
    return O


@pytest.fixture(autouse=True)
def _torch_hip_first(request):
    """GPU tests: torch's HIP runtime (it bundles its own) is initialised once, before the first
    test touches the device through libsm_hip.so, as the test order of the whole suite does anyway
    (test_gpu_batch.py precedes the fixture tests); a late first torch.cuda call in a subset run
    once failed with "No HIP GPUs are available" after many of our contexts had come and gone."""
    if request.node.get_closest_marker("gpu") is not None and not getattr(_torch_hip_first, "done", False):
        _torch_hip_first.done = True
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    yield
