"""In-process repeatability of fit + posterior variance: REPS fits of the same data, each
followed by the variance at Q queries, compared bitwise with the first.  Prints the repetitions
that differ (count of differing entries, max relative difference).  Usage:
det_loop.py N Q REPS [f32|f64 [SAVE_PREFIX]]  (the first two repetitions saved as SAVE_PREFIX_repR.npy:
variances then means)"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import gpr_amd  # noqa: E402
from gpr_amd.synth import make_data, make_queries  # noqa: E402

n, q, reps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
dt = np.float32 if len(sys.argv) > 4 and sys.argv[4] == "f32" else np.float64
ctx = gpr_amd.Context(0)
X, Y = make_data(n, 8)
Xq = make_queries(q, 8)
M = gpr_amd.Model(ctx, dt)
M.set_data(X, Y)
M.set_kernel("GaussianKernel(1.3,1,)")
M.set_noise(0.5)
ref = None
bad = 0
for r in range(reps):
    M.fit()
    v = np.asarray(M.posterior_cov(Xq, Xq))
    mu = np.asarray(M.predict(Xq)) if hasattr(M, "predict") else v
    parts = [v.ravel(), np.asarray(mu).ravel()]
    if os.environ.get("DET_LML"):  # also the LML + gradient (factor with the inverse riding along)
        lv, lg, ld = M.lml(grad=True)
        parts.append(np.concatenate([[lv, ld], np.asarray(lg, np.float64).ravel()]))
    out = np.concatenate(parts)
    if r < 2 and len(sys.argv) > 5:
        np.save(f"{sys.argv[5]}_rep{r}.npy", out)
    if ref is None:
        ref = out
        continue
    if not np.array_equal(out, ref):
        d = np.abs(out - ref)
        bad += 1
        idx = np.nonzero(d)[0]
        print(f"rep {r}: ndiff {len(idx)} (variance {int((idx < q).sum())}, mean {int((idx >= q).sum())}) "
              f"maxrel {float((d / np.maximum(np.abs(ref), 1e-300)).max()):.3e} first {idx[:6].tolist()} "
              f"last {idx[-3:].tolist()}", flush=True)
print(f"N {n} Q {q} {np.dtype(dt).name}: {bad} of {reps - 1} repetitions differ", flush=True)
