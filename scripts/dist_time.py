"""Timing of the storage-sharded fit at C3 size: single-GPU engine, virtual ranks g = 1, 2, 4
on one GPU (each rank on its own CU share), and the RCCL transport on a one-rank communicator.
Usage: python scripts/dist_time.py [N] [steps] [modes...]   (modes: single v1 v2 v4 rccl1)"""
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
X, Y = make_data(n, C3["d"], 1)
ref = None
for mode in modes:
    if mode == "single":
        ctx = gpr_amd.Context(0)
    elif mode.startswith("v"):
        ctx = gpr_amd.Context(0, virtual=int(mode[1:]))
    else:
        ctx = gpr_amd.Context(0, dist=(0, 1, gpr_amd.unique_id()))
    M = gpr_amd.Model(ctx, np.float64)
    M.set_data(X, Y)
    M.set_kernel(C3["kernel"])
    M.set_noise(C3["sigma"])
    flags = gpr_amd.gprx.FIT_DISTRIBUTED if mode == "rccl1" else 0
    for _ in range(2):
        M.fit(flags)
    t0 = time.perf_counter()
    for _ in range(steps):
        info = M.fit(flags)
    dt = (time.perf_counter() - t0) / steps
    a = M.alpha()
    if ref is None:
        ref = a
    err = float(np.max(np.abs(a - ref)) / np.max(np.abs(ref)))
    print(f"{mode:7s} N={n}: {1e3 * dt:8.2f} ms/fit  {1 / dt:7.2f} fits/s  logdet {info.logdet:.10e}  "
          f"alpha vs first {err:.2e}", flush=True)
    M.close()
    ctx.close()
