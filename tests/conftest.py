import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests proper")


def _ensure_built():
    lib = os.path.join(ROOT, "dynosam_amd", "lib")
    need = [os.path.join(lib, "libdynohip.so"), os.path.join(lib, "libdynosynth.so"),
            os.path.join(ROOT, "oracle", "build", "liboracle.so")]
    if not all(os.path.exists(p) for p in need):
        import __graft_entry__
        __graft_entry__.build()


_ensure_built()


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test requested but no HIP device is visible")
    return True
