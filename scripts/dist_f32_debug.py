import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import gpr_amd
from tests.helpers import make_data
from oracle import oracle as O
RQK = "RationalQuadraticKernel(1.1,0.6,1.5,)"
n, d, sigma = 1500, 5, 0.6
X, Y = make_data(n, d, 2)
X32, Y32 = X.astype(np.float32), Y.astype(np.float32)
rq32 = "RationalQuadraticKernel({},{},{},)".format(*[repr(float(np.float32(v))) for v in (1.1, 0.6, 1.5)])
a64, _ = O.fit(rq32, X32.astype(np.float64), Y32.astype(np.float64), float(np.float32(sigma)), want_core=False)
for steps in ("3",):
    os.environ["GPRX_REFINE_STEPS"] = steps
    for g in (0, 2, 3):
        for m in (1, 2):
            ctx = gpr_amd.Context(0, virtual=g) if g else gpr_amd.Context(0)
            M = gpr_amd.Model(ctx, np.float32)
            M.set_data(X32, Y32[:, :m].copy())
            M.set_kernel(RQK)
            M.set_noise(sigma)
            info = M.fit()
            a = M.alpha().astype(np.float64)
            errs = [float(np.max(np.abs(a[:, c] - a64[:, c])) / np.max(np.abs(a64[:, c]))) for c in range(m)]
            print(json.dumps({"refine_steps_env": steps, "g": g, "m": m, "col_err": errs, "steps": info.refine_steps,
                              "delta": info.refine_delta}), flush=True)
            M.close()
            ctx.close()
