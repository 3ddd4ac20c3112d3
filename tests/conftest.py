import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm device); run with -m gpu")


def gpu_available() -> bool:
    import torch
    return torch.cuda.is_available()


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from quantized_vit_amd import build
    build.build()
    return torch.device("cuda:0")
