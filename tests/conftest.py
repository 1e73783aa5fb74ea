import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: multi-process / long-running test")


def _native_built():
    import glob
    pkg = os.path.join(ROOT, "distributed_llms_amd")
    return glob.glob(os.path.join(pkg, "_C_runtime*.so")) and glob.glob(os.path.join(pkg, "_C_kernels*.so"))


@pytest.fixture(scope="session", autouse=True)
def _ensure_native_built():
    """Build the in-tree extensions once if they are missing (hipcc cross-compiles on CPU)."""
    if not _native_built():
        from distributed_llms_amd.csrc import build
        build.build_all()
    yield


@pytest.fixture
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda")
