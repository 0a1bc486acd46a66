import os
import sys

import pytest

# The distributed fit's virtual ranks (tests/test_gpu_dist.py) run a persistent launch per rank
# next to two transport streams: every stream needs a hardware queue of its own, or a
# transport command queued behind a persistent launch on a shared queue could never run
# (HIP's default is 4 queues per process; gpurun allows up to 32).  Set before HIP starts.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libgprx on cuda:0)")


@pytest.fixture(scope="session")
def ctx():
    import gpr_amd
    c = gpr_amd.Context(0)
    yield c
    c.close()
