#!/usr/bin/env python3
"""Fit throughput on BASELINE.json's other dense configurations, one GPU.

* C2 (configs[1]): N=4096, d=16, GaussianKernel(1,1), sigma=0.1, fp64.
* C4 (configs[3]): N=32768, d=32, RationalQuadraticKernel(1,0.3,1), sigma=1.0, fp32
  (quoted on 8 GPUs; this is the single-GPU fit the replicas mode runs per rank).

One step = one full fit (covariance build + Cholesky + regression solve; for fp32 also the
fp64 iterative refinement of alpha, the reference inverting fp32 GPs in double,
include/LAPACKUtils.h:85-97), X and Y resident on the device before the timed region.  fp64
configurations also check the residual ||(K + s^2 I) alpha - Y||_inf / ||Y||_inf with K from
the separately parity-tested kernel-matrix path; fp32 ones compare alpha with the fp64 fit
of the same data (BASELINE tolerance 1e-3).  Prints one JSON line per configuration.

    python scripts/bench_configs.py [--steps 5] [--only C4]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK = {"f64": 78.6, "f32": 157.3}  # dense MFMA TFLOP/s, MI355X_MICROARCH.md


def run(name, cfg, steps, warmup):
    import gpr_amd
    from gpr_amd.synth import make_data
    dtype = np.float64 if cfg["dtype"] == "f64" else np.float32
    n, d = cfg["n"], cfg["d"]
    X, Y = make_data(n, d, cfg["m"])
    ctx = gpr_amd.Context(0)
    M = gpr_amd.Model(ctx, dtype)
    M.set_data(X.astype(dtype), Y.astype(dtype))
    M.set_kernel(cfg["kernel"])
    M.set_noise(cfg["sigma"])
    for _ in range(warmup):
        M.fit()
    ph = np.zeros(4)
    t0 = time.perf_counter()
    for _ in range(steps):
        info = M.fit()
        ph += (info.ms_build, info.ms_factor, info.ms_solve, info.ms_refine)
    dt = (time.perf_counter() - t0) / steps
    ph /= steps
    alpha = M.alpha().astype(np.float64)
    check = {}
    if dtype == np.float64:
        K = ctx.kernel_matrix(cfg["kernel"], X, dtype=dtype)
        K[np.diag_indices(n)] += cfg["sigma"] ** 2
        r = K @ alpha - Y
        del K
        check["residual"] = float(np.max(np.abs(r)) / np.max(np.abs(Y)))
    else:
        M64 = gpr_amd.Model(ctx, np.float64)
        M64.set_data(X.astype(dtype).astype(np.float64), Y.astype(dtype).astype(np.float64))
        M64.set_kernel(cfg["kernel"])
        M64.set_noise(cfg["sigma"])
        M64.fit()
        a64 = M64.alpha()
        check["alpha_vs_f64_fit"] = float(np.max(np.abs(alpha - a64)) / np.max(np.abs(a64)))
        check["refine_steps"] = int(info.refine_steps)
        check["refine_delta"] = float(info.refine_delta)
        M64.close()
    tflops = n ** 3 / 3.0 / (ph[1] * 1e-3) / 1e12
    out = {
        "config": name, "n": n, "d": d, "kernel": cfg["kernel"], "dtype": cfg["dtype"],
        "fits_per_s": 1.0 / dt, "ms_per_fit_wall": dt * 1e3,
        "ms_build": ph[0], "ms_factor": ph[1], "ms_solve": ph[2], "ms_refine": ph[3],
        "factor_tflops": tflops, "factor_frac_of_peak": tflops / PEAK[cfg["dtype"]],
        "info": int(info.info), "logdet": float(info.logdet), **check,
    }
    print(json.dumps(out), flush=True)
    M.close()
    ctx.close()
    return out


def main():
    from gpr_amd.synth import C2, C4
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    tol = {"f64": 1e-10, "f32": 1e-3}
    ok = True
    for name, cfg in (("C2", C2), ("C4", C4)):
        if a.only and a.only != name:
            continue
        o = run(name, cfg, a.steps, a.warmup)
        ok &= o["info"] == 0 and o.get("residual", o.get("alpha_vs_f64_fit")) <= tol[cfg["dtype"]]
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
