import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libxcodec_hip.so)")
    config.addinivalue_line("markers", "slow: long-running case")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def gpu_ctx():
    import wanproxy_amd as w
    if w.device_count() < 1:
        pytest.fail("no GPU visible but a gpu-marked test ran")
    ctx = w.Context(0)
    yield ctx  # released (after its caches) by wanproxy_amd.xcodec's exit teardown
