import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")


@pytest.fixture(scope="session", autouse=True)
def _native_runtime():
    # The host runtime .so is git-ignored: build it once per session (seconds, incremental).
    from mihvd import _native

    _native.runtime()
    yield


@pytest.fixture
def hvd_single():
    """A single-process mihvd world (gloo on CPU, RCCL when a GPU is visible)."""
    import mihvd.torch as hvd

    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT", "OMPI_COMM_WORLD_RANK"):
        os.environ.pop(k, None)
    hvd.init()
    yield hvd
    hvd.shutdown()
