"""Debugging aid: which stage of a (sharded) fit reads unwritten memory.  Run with GPRX_POISON=1
(fresh device buffers filled with finite garbage).  Prints alpha vs the oracle without and with
the fp32 refinement, and the core matrix (K + s^2 I)^{-1} from the (gathered) factor."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import gpr_amd  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.helpers import make_data, relerr  # noqa: E402

ks = sys.argv[1] if len(sys.argv) > 1 else "SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))"
n, d, sigma = 1100, 4, 0.6
X, Y = make_data(n, d, 1)
for dt in (np.float64, np.float32):
    Xt, Yt = X.astype(dt), Y.astype(dt)
    a_ref, _ = O.fit(ks, Xt, Yt, sigma, dt if dt == np.float32 else np.float64, want_core=False)
    K = O.kernel_matrix(ks, Xt.astype(np.float64)) + sigma * sigma * np.eye(n)
    Cref = np.linalg.inv(K)
    for g in (0, 1, 2):
        for steps in ("0", "3"):
            os.environ["GPRX_REFINE_STEPS"] = steps
            ctx = gpr_amd.Context(0, virtual=g) if g else gpr_amd.Context(0)
            M = gpr_amd.Model(ctx, dt)
            M.set_data(Xt, Yt)
            M.set_kernel(ks)
            M.set_noise(sigma)
            info = M.fit()
            line = {"dtype": np.dtype(dt).name, "g": g, "steps": steps, "alpha_err": relerr(M.alpha(), a_ref),
                    "logdet": info.logdet, "logdet_ref": float(np.linalg.slogdet(K)[1])}
            if steps == "0":
                Cm = M.core_matrix()
                line["core_err"] = float(np.max(np.abs(Cm - Cref)) / np.max(np.abs(Cref)))
            print(json.dumps(line), flush=True)
            M.close()
            ctx.close()
