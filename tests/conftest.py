import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "map-reduced-approach-for-vietnamese-long-document-summarization_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmapsum.so on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def has_gpu():
    import torch
    return torch.cuda.is_available()
