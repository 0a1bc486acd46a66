"""C2 fit timeline: K fits of N=4096 d=16 Gaussian back to back (the bench's C2 leg), wall time
per fit, for reading with a rocprofv3 kernel trace of the same run (the gaps between one fit's
kernels and between fits are the host-side share of C2's ms per fit).
usage: python scripts/c2_timeline.py [K] [stats 0/1]"""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import gpr_amd  # noqa: E402
from gpr_amd.synth import C2, make_data  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 50
stats = len(sys.argv) > 2 and sys.argv[2] == "1"
ctx = gpr_amd.Context(0)
X, Y = make_data(C2["n"], C2["d"], C2["m"])
M = gpr_amd.Model(ctx, np.float64)
M.set_data(X, Y)
M.set_kernel(C2["kernel"])
M.set_noise(C2["sigma"])
for _ in range(3):
    M.fit()
if stats:
    ctx.set_stats(True)
t0 = time.perf_counter()
for _ in range(K):
    M.fit()
el = time.perf_counter() - t0
print({"fits": K, "ms_per_fit": 1e3 * el / K, "fits_per_s": K / el, "stats": stats}, flush=True)
M.close()
ctx.close()
