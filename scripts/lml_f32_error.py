"""fp32 LML + gradient error: the fp32 model's LML (fp32 factor with the inverse riding along)
against the fp64 model on the same float data (validated against the oracle at 1e-6) and, at
N <= 4096, against the oracle's fp32 path (the reference: K in float, inverted in double)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import gpr_amd  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.helpers import make_data  # noqa: E402

C3K = "SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))"
ctx = gpr_amd.Context(0)
for n, d, sigma in [(4096, 32, 1.0), (16384, 32, 1.0)]:
    X, Y = make_data(n, d, 1)
    X32, Y32 = X.astype(np.float32), Y.astype(np.float32)
    res = {"n": n, "d": d}
    out = {}
    for dt in (np.float32, np.float64):
        M = gpr_amd.Model(ctx, dt)
        M.set_data(X32.astype(dt), Y32.astype(dt))
        M.set_kernel(C3K)
        M.set_noise(sigma)
        M.lml(grad=True)
        t0 = time.perf_counter()
        v, g, ld = M.lml(grad=True)
        out[np.dtype(dt).name] = (v, np.array(g), time.perf_counter() - t0)
        M.close()
    v32, g32, t32 = out["float32"]
    v64, g64, t64 = out["float64"]
    res.update(ms_f32=1e3 * t32, ms_f64=1e3 * t64, value_relerr_vs_f64=abs(v32 - v64) / abs(v64),
               grad_relerr_vs_f64=float(np.max(np.abs(g32 - g64)) / np.max(np.abs(g64))),
               grad_f32=list(map(float, g32)), grad_f64=list(map(float, g64)))
    if n <= 4096:
        vr, gr, _, _ = O.lml(C3K, X32, Y32, sigma, np.float32)
        res.update(grad_relerr_vs_oracle_f32=float(np.max(np.abs(g32 - np.array(gr))) / np.max(np.abs(np.array(gr)))),
                   value_relerr_vs_oracle_f32=abs(v32 - vr) / abs(vr))
    print(json.dumps(res, default=float), flush=True)
ctx.close()
