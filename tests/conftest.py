import os
import sys

import pytest

# The reactive transport runs one HIP stream per peer; with several ranks in
# one process (GPU loopback tests) the streams must not share hardware queues
# (a stream parked on a wait would block unrelated streams).  HIP reads this at
# its first call, so set it before anything touches the GPU.  (<= 32 allowed.)
os.environ["GPU_MAX_HW_QUEUES"] = "32"  # the box exports 4

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: longer-running test")


def _has_gpu() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def native():
    from akka_allreduce_amd import _native_loader

    return _native_loader.load()


@pytest.fixture(autouse=True)
def _stream_race_check():
    """With AKKA_RACECHECK=1 (CPU), every simulated cluster a test built must
    end race-free: the engine's own stream/event ordering is checked in every
    simulator test, not only in tests/test_racecheck.py."""
    yield
    if os.environ.get("AKKA_RACECHECK", "0") in ("", "0"):
        return
    from akka_allreduce_amd.parallel.sim import LIVE_CLUSTERS

    reports = [m for c in list(LIVE_CLUSTERS) for m in c.race_reports()]
    LIVE_CLUSTERS.clear()
    assert not reports, "stream races:\n" + "\n".join(reports[:10])
