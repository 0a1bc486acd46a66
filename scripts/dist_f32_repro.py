"""Debugging aid: the fp32 m = 2 sharded fit after a large fit in the same process."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import gpr_amd  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.helpers import make_data  # noqa: E402

RQK = "RationalQuadraticKernel(1.1,0.6,1.5,)"
C4K = "RationalQuadraticKernel(1,1,1,)"
big = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
if big:
    X, Y = make_data(big, 32, 1)
    mode = sys.argv[2] if len(sys.argv) > 2 else "rccl"
    c = gpr_amd.Context(0, dist=(0, 1, gpr_amd.unique_id())) if mode == "rccl" else gpr_amd.Context(0, virtual=2)
    M = gpr_amd.Model(c, np.float32)
    M.set_data(X.astype(np.float32), Y.astype(np.float32))
    M.set_kernel(C4K)
    M.set_noise(1.0)
    M.fit(gpr_amd.gprx.FIT_DISTRIBUTED if mode == "rccl" else 0)
    M.close()
    c.close()
    print("big fit done", flush=True)
n, d, sigma = 1500, 5, 0.6
X, Y = make_data(n, d, 2)
X32, Y32 = X.astype(np.float32), Y.astype(np.float32)
rq32 = "RationalQuadraticKernel({},{},{},)".format(*[repr(float(np.float32(v))) for v in (1.1, 0.6, 1.5)])
a64, _ = O.fit(rq32, X32.astype(np.float64), Y32.astype(np.float64), float(np.float32(sigma)), want_core=False)
for rep in range(4):
    for steps in ("0", "3"):
        os.environ["GPRX_REFINE_STEPS"] = steps
        ctx = gpr_amd.Context(0, virtual=2)
        M = gpr_amd.Model(ctx, np.float32)
        M.set_data(X32, Y32)
        M.set_kernel(RQK)
        M.set_noise(sigma)
        info = M.fit()
        a = M.alpha().astype(np.float64)
        err = [float(np.max(np.abs(a[:, c] - a64[:, c])) / np.max(np.abs(a64[:, c]))) for c in range(2)]
        bad = int(np.argmax(np.abs(a[:, 0] - a64[:, 0])))
        print(json.dumps({"rep": rep, "steps_env": steps, "col_err": err, "steps": info.refine_steps,
                          "delta": info.refine_delta, "worst_row": bad, "worst": [float(a[bad, 0]), float(a64[bad, 0])],
                          "nbad": int(np.sum(np.abs(a[:, 0] - a64[:, 0]) > 1e-3))}), flush=True)
        M.close()
        ctx.close()
