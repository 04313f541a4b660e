import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libedt_sync.so")
    config.addinivalue_line("markers", "slow: multi-process or large-size test")


@pytest.fixture(scope="session")
def golden():
    from tests.golden_data import Golden
    return Golden()


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as o
    o.build()
    return o


@pytest.fixture(autouse=True, scope="module")
def _release_device_memory():
    """After each test module: collect cycles and hand the caching allocator's blocks back, so a
    module that filled HBM (the 7B populations) cannot starve the next one."""
    yield
    import gc
    gc.collect()
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
    except Exception:       # noqa: BLE001 - best effort, never fails a test
        pass
