import os
import sys

import pytest

# (The GPU tests run with the box's default hardware-queue count, the setting bench.py runs
# under: the sharded fit's virtual ranks each launch on a CU-masked stream of their own, and
# the exchange is the kernels' own stores -- no transport stream that could queue behind them.)

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
