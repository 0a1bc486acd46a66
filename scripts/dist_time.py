"""Timing of the storage-sharded fit: the single-GPU engine, virtual ranks g = 1..8 on one GPU
(each rank on its own CU share: the whole chip does the same work as one rank would, so the
ideal is the single-GPU time plus the exchange), and the one-rank RCCL context.
Usage: python scripts/dist_time.py [N] [steps] [modes...]
  modes: single v1 v2 v4 rccl1, and lml:<mode> for the LML + gradient (sharded potri)
  GPRX_DIST_DTYPE=f32 runs fp32 (with the sharded fp64 refinement)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import gpr_amd  # noqa: E402
from gpr_amd.synth import C3, make_data  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else C3["n"]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
modes = sys.argv[3:] or ["single", "v1", "v2", "rccl1"]
dt_ = np.float32 if os.environ.get("GPRX_DIST_DTYPE") == "f32" else np.float64
kern = os.environ.get("GPRX_DIST_KERNEL", C3["kernel"])
X, Y = make_data(n, C3["d"], 1)
X, Y = X.astype(dt_), Y.astype(dt_)
ref = None
for mode in modes:
    lml = mode.startswith("lml:")
    base = mode[4:] if lml else mode
    if base == "single":
        ctx = gpr_amd.Context(0)
    elif base.startswith("v"):
        ctx = gpr_amd.Context(0, virtual=int(base[1:]))
    else:
        ctx = gpr_amd.Context(0, dist=(0, 1, gpr_amd.unique_id()))
    M = gpr_amd.Model(ctx, dt_)
    M.set_data(X, Y)
    M.set_kernel(kern)
    M.set_noise(C3["sigma"])
    flags = gpr_amd.gprx.FIT_DISTRIBUTED if base == "rccl1" else 0
    if lml:
        for _ in range(2):
            M.lml(grad=True, distributed=(base != "single"))
        t0 = time.perf_counter()
        for _ in range(steps):
            v, g, ld = M.lml(grad=True, distributed=(base != "single"))
        dt = (time.perf_counter() - t0) / steps
        print(json.dumps({"mode": mode, "n": n, "ms_lml_grad": 1e3 * dt, "value": v, "grad": list(g)}), flush=True)
    else:
        for _ in range(2):
            M.fit(flags)
        t0 = time.perf_counter()
        for _ in range(steps):
            info = M.fit(flags)
        dt = (time.perf_counter() - t0) / steps
        a = M.alpha()
        if ref is None:
            ref = a
        err = float(np.max(np.abs(a.astype(np.float64) - ref)) / np.max(np.abs(ref)))
        line = {"mode": mode, "n": n, "dtype": np.dtype(dt_).name, "ms_per_fit": 1e3 * dt, "fits_per_s": 1 / dt,
                "ms_factor_kernel": info.ms_factor, "ms_solve": info.ms_solve, "ms_refine": info.ms_refine,
                "logdet": info.logdet, "alpha_vs_first": err}
        if base != "single":
            line["dist"] = M.dist_info()
        print(json.dumps(line), flush=True)
    M.close()
    ctx.close()
