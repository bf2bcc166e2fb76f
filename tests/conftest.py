import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box with -m gpu)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


_TORCH_HIP = False


def pytest_runtest_setup(item):
    """Before the first GPU test of the session: initialise the HIP runtime through torch, so that torch (used
    by some GPU tests for device buffers) owns the runtime before libkad.so creates its contexts — torch's own
    lazy init fails with "No HIP GPUs are available" once libkad.so has initialised HIP first in the process."""
    global _TORCH_HIP
    if _TORCH_HIP or item.get_closest_marker("gpu") is None:
        return
    _TORCH_HIP = True
    try:
        import torch
    except ImportError:
        return
    if torch.cuda.is_available():
        torch.cuda.init()
