import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C-ABI)")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    oracle.lib()
    return oracle


_torch_cuda_ready = False


def pytest_runtest_setup(item):
    """Before the first GPU test: initialise torch's HIP runtime.  torch's wheel bundles its own
    libamdhip64 beside the /opt/rocm one libtfusion_hip.so links; torch's fails to find a device
    when it initialises after the other, so the tests that render frames with torch on the GPU
    (bench.orbit_frames / walk_frames) need it to go first, as bench.py's own import order does."""
    global _torch_cuda_ready
    if _torch_cuda_ready or item.get_closest_marker("gpu") is None:
        return
    _torch_cuda_ready = True
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass
