import os
import sys
from hashlib import sha256

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "deep-attention-visual-odometry_amd")
for p in (REPO, SRC):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")


@pytest.fixture()
def fixed_random_seed(request) -> int:
    """Same per-test seed as the reference's tests/conftest.py:21-23 (with the
    byteorder spelled out so it also works on Python 3.10)."""
    return abs(int.from_bytes(sha256(request.node.name.encode("utf-8")).digest()[:8], "big"))


@pytest.fixture(scope="session")
def device():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda", 0)


@pytest.fixture()
def overrides():
    """overrides(name, value): one of the library's launch choices (or the Python side's generic-loop
    switches) for this test, through _native.set_debug_override; every override is cleared afterwards.
    The library never reads them from the environment."""
    from deep_attention_visual_odometry_amd import _native

    yield _native.set_debug_override
    _native.clear_debug_overrides()
