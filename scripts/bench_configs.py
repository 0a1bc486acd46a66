#!/usr/bin/env python3
"""Fit throughput on BASELINE.json's other dense configurations, one GPU.

* C2 (configs[1]): N=4096, d=16, GaussianKernel(1,1), sigma=0.1, fp64.
* C4 (configs[3]): N=32768, d=32, RationalQuadraticKernel(1,0.3,1), sigma=1.0, fp32
  (quoted on 8 GPUs; this is the single-GPU fit the replicas mode runs per rank).

One step = one full fit (covariance build + Cholesky + regression solve), X and Y resident
on the device before the timed region.  Each configuration also checks the size-independent
residual property ||(K + s^2 I) alpha - Y||_inf / ||Y||_inf, with K from the separately
parity-tested kernel-matrix path.  Prints one JSON line per configuration.

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
    ph = np.zeros(3)
    t0 = time.perf_counter()
    for _ in range(steps):
        info = M.fit()
        ph += (info.ms_build, info.ms_factor, info.ms_solve)
    dt = (time.perf_counter() - t0) / steps
    ph /= steps
    alpha = M.alpha().astype(np.float64)
    K = ctx.kernel_matrix(cfg["kernel"], X.astype(dtype), dtype=dtype)
    K[np.diag_indices(n)] += dtype(cfg["sigma"] ** 2)
    r = K.astype(np.float64) @ alpha - Y
    del K
    res = float(np.max(np.abs(r)) / np.max(np.abs(Y)))
    tflops = n ** 3 / 3.0 / (ph[1] * 1e-3) / 1e12
    out = {
        "config": name, "n": n, "d": d, "kernel": cfg["kernel"], "dtype": cfg["dtype"],
        "fits_per_s": 1.0 / dt, "ms_per_fit_wall": dt * 1e3,
        "ms_build": ph[0], "ms_factor": ph[1], "ms_solve": ph[2],
        "factor_tflops": tflops, "factor_frac_of_peak": tflops / PEAK[cfg["dtype"]],
        "residual": res, "info": int(info.info), "logdet": float(info.logdet),
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
        ok &= o["info"] == 0 and o["residual"] <= tol[cfg["dtype"]]
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
