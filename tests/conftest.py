import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "image-caption_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture
def set_knob():
    """set_knob(name, value): a library run-time switch (capgen_set_knob, name without CAPGEN_) for the
    test; every switch it touched is restored afterwards."""
    from capgen import _lib
    saved = {}

    def _set(name, value):
        old = _lib.set_knob(name, int(value))
        saved.setdefault(name, old)

    yield _set
    for name, old in saved.items():
        _lib.set_knob(name, old)
