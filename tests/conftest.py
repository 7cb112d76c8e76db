import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "semantic-bundle-adjustment-colmap_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmi_ba.so on cuda:0)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


def has_gpu():
    try:
        import mi_ba
        return mi_ba.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    import mi_ba
    mi_ba.load()
    if mi_ba.device_count() == 0:
        pytest.fail("gpu-marked test without a visible MI355X (product has no CPU fallback)")
    return True
