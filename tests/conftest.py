import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session", autouse=True)
def _native_lib():
    from distributed_machine_learning_project_amd import build
    build.build(engine=False)
    yield


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
