import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "depth-map-fusion-utils_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity tests through the C ABI")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    # torch's HIP runtime must be the process's first: libdmf.so shares it (a libdmf call
    # before torch's CUDA init left torch with "No HIP GPUs are available" when a test file
    # that starts with libdmf-only tests ran on its own)
    import torch  # noqa: F401
    if torch.cuda.device_count() > 0:  # counting devices does not initialise the GPU
        torch.cuda.init()


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O
