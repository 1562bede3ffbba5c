import os
import sys
import warnings

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

warnings.filterwarnings("ignore", message="The PyTorch API of MaskedTensors")
warnings.filterwarnings("ignore", message="It is not recommended to create a MaskedTensor")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def device():
    """
    The GPU for `-m gpu` tests. No skip: on a GPU box a missing device or library is a failure.
    """
    import torch
    from mininf_amd import _native
    assert torch.cuda.is_available(), "gpu tests need a ROCm device"
    _native.lib()
    return torch.device("cuda:0")


@pytest.fixture(autouse=True)
def _clean_contexts():
    """
    Contexts are process-global (reference core.py:25); make sure a failing test cannot leak one.
    """
    yield
    from mininf_amd.core import SingletonContextMixin
    SingletonContextMixin.INSTANCES.clear()


def golden(name):
    import numpy as np
    return np.load(os.path.join(ROOT, "tests", "golden", name))
