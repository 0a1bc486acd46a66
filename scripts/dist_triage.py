"""Correctness sweep of the sharded fit over virtual ranks / windows / groupings: alpha and
log det against the single-GPU fit.  Usage: python scripts/dist_triage.py N g[,g..] [ww|0] [gb|0]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import gpr_amd  # noqa: E402
from gpr_amd.synth import C3, make_data  # noqa: E402

n = int(sys.argv[1])
gs = [int(x) for x in sys.argv[2].split(",")]
ww = int(sys.argv[3]) if len(sys.argv) > 3 else 0
gb = int(sys.argv[4]) if len(sys.argv) > 4 else 0
if ww:
    os.environ["GPRX_DIST_WINDOW"] = str(ww)
if gb:
    os.environ["GPRX_DIST_GROUP"] = str(gb)
X, Y = make_data(n, 32, 1)
c = gpr_amd.Context(0)
M = gpr_amd.Model(c, np.float64)
M.set_data(X, Y)
M.set_kernel(C3["kernel"])
M.set_noise(C3["sigma"])
i0 = M.fit()
a0 = M.alpha()
M.close()
c.close()
for g in gs:
    v = gpr_amd.Context(0, virtual=g)
    M = gpr_amd.Model(v, np.float64)
    M.set_data(X, Y)
    M.set_kernel(C3["kernel"])
    M.set_noise(C3["sigma"])
    errs = []
    for _ in range(3):
        info = M.fit()
        errs.append(float(np.max(np.abs(M.alpha() - a0)) / np.max(np.abs(a0))))
    print(json.dumps({"n": n, "g": g, "err": errs, "dlogdet": info.logdet - i0.logdet, "dist": M.dist_info()}), flush=True)
    M.close()
    v.close()
