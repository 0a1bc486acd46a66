"""Log-marginal likelihood + gradient at C3 (BASELINE.json configs[2]): device time per
phase (ctx stats) after one warm-up call.  python scripts/lml_time.py [n]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import gpr_amd
from gpr_amd.synth import C3, make_data

n = int(sys.argv[1]) if len(sys.argv) > 1 else C3["n"]
ctx = gpr_amd.Context(0)
X, Y = make_data(n, C3["d"], C3["m"])
M = gpr_amd.Model(ctx, np.float64)
M.set_data(X, Y)
M.set_kernel(C3["kernel"])
M.set_noise(C3["sigma"])
M.lml(grad=True)
ctx.set_stats(True)
t0 = time.perf_counter()
v = M.lml(grad=True)
dt = time.perf_counter() - t0
st = ctx.stats()
ctx.set_stats(False)
print(json.dumps({"n": n, "wall_ms_lml_grad": 1e3 * dt, "lml": str(v)[:200],
                  "phases_ms": {k: round(s["ms"], 3) for k, s in st.items()}}, indent=1))
