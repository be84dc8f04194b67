import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, HERE, os.path.join(HERE, "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and librfa.so")


@pytest.fixture(scope="session")
def rfa():
    """librfa on a real device; fails loudly (no CPU fallback) when absent."""
    import rfanalyzer_amd

    n = rfanalyzer_amd.device_count()
    assert n > 0, "no HIP device visible to librfa"
    return rfanalyzer_amd
