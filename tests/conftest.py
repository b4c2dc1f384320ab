import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

PKG_NAME = "pointcloud-segmentation-attention_amd"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


@pytest.fixture(scope="session")
def pn2():
    return importlib.import_module(PKG_NAME)


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle
    return oracle


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
