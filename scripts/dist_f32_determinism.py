"""Debugging aid: is the fp32 refinement (single-GPU / sharded) bitwise repeatable?"""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import gpr_amd  # noqa: E402
from tests.helpers import make_data  # noqa: E402

RQK = "RationalQuadraticKernel(1.1,0.6,1.5,)"
n, d, sigma = 1500, 5, 0.6
X, Y = make_data(n, d, 2)
X32, Y32 = X.astype(np.float32), Y.astype(np.float32)
for g in (0, 1, 2):
    for steps in ("1", "2", "3"):
        os.environ["GPRX_REFINE_STEPS"] = steps
        hs = []
        ctx = gpr_amd.Context(0, virtual=g) if g else gpr_amd.Context(0)
        M = gpr_amd.Model(ctx, np.float32)
        M.set_data(X32, Y32)
        M.set_kernel(RQK)
        M.set_noise(sigma)
        for rep in range(6):
            info = M.fit()
            hs.append((hashlib.sha1(M.alpha().tobytes()).hexdigest()[:10], info.refine_steps, "%.3e" % info.refine_delta))
        print(json.dumps({"g": g, "steps": steps, "distinct": len(set(h[0] for h in hs)), "runs": hs}), flush=True)
        M.close()
        ctx.close()
