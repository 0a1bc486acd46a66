"""Debug driver for the distributed fit on virtual ranks: one fit, the issue loop's end state
printed by libgprx (GPRX_DIST_DEBUG=1)."""
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
os.environ.setdefault("GPRX_DIST_DEBUG", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import gpr_amd  # noqa: E402
from gpr_amd.synth import make_data  # noqa: E402

g = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n = int(sys.argv[2]) if len(sys.argv) > 2 else 700
ks = sys.argv[3] if len(sys.argv) > 3 else "SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))"
X, Y = make_data(n, 5, 1)
ctx = gpr_amd.Context(0, virtual=g)
M = gpr_amd.Model(ctx, np.float64)
M.set_data(X, Y)
M.set_kernel(ks)
M.set_noise(0.5)
t = time.time()
try:
    info = M.fit()
    print("fit ok", time.time() - t, info.logdet, flush=True)
except Exception as e:
    print("fit failed", time.time() - t, e, flush=True)
