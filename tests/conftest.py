import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP engine)")
    config.addinivalue_line("markers", "slow: long-running (full-size model) test")


@pytest.fixture(scope="session")
def gpu_lib():
    """The engine library; GPU tests must run the native HIP path (no fallback)."""
    from blama_amd import engine
    return engine.lib()
