"""pytest configuration: `gpu` marker, import paths, shared fixtures.

`-m "not gpu"` runs everywhere (oracle vs golden vectors, host preprocessing,
C-ABI symbol checks, gloo multi-process plumbing); `-m gpu` runs the parity
tests proper on an MI355X through the C ABI.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "spmm-denseblock_amd"), os.path.join(ROOT, "tests"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests")


@pytest.fixture(scope="session")
def oracle():
    from helpers import load_oracle
    return load_oracle()


@pytest.fixture(scope="session")
def golden():
    from helpers import load_golden
    return load_golden()


@pytest.fixture(scope="session")
def device():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no HIP device is visible")
    return torch.device("cuda", 0)
