"""Run-to-run determinism of the posterior covariance path (test_gpu_tiles.py's
test_posterior_tall_gemms_match_128_tiles child) under environment variants: each variant
in its own process, the outputs compared bitwise.  Usage: det_check.py OUTDIR VAR... where
VAR is "-" or comma-joined NAME=VALUE settings."""
import os
import subprocess
import sys

import numpy as np

_here = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(_here, ".."), os.path.join(_here, "..", "tests")]
from test_gpu_tiles import _TALL_CHILD  # noqa: E402

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = sys.argv[1]
os.makedirs(out, exist_ok=True)
res = []
for q, v in enumerate(sys.argv[2:]):
    env = dict(os.environ)
    if v != "-":
        env.update(kv.split("=", 1) for kv in v.split(","))
    f = os.path.join(out, f"det_{q}.npy")
    r = subprocess.run([sys.executable, "-c", _TALL_CHILD, root, f], env=env, capture_output=True, text=True,
                       timeout=240)
    if r.returncode != 0:
        print(r.stderr[-2000:])
        sys.exit(r.returncode)
    res.append((v, np.load(f)))
    print(f"{q} {v} done", flush=True)
for q, (v, a) in enumerate(res):
    d = np.abs(a - res[0][1])
    print(f"{q} {v}: equal={np.array_equal(a, res[0][1])} ndiff={int((d > 0).sum())} maxrel={float((d / np.abs(res[0][1])).max()):.3e}")
