"""Timeline of one chained back substitution (GPRX_BS_TRACE) after a C3 fit: per block the
time from alpha_{k+1} published to alpha_k published (the chain step), and how late the
non-critical tiles finish relative to alpha_{k+1}."""
import ctypes, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("GPRX_BS_TRACE", "1")
import numpy as np
import gpr_amd
from gpr_amd.gprx import lib
from gpr_amd.synth import C3, make_data

L = lib()
L.gprx_dev_bs_trace.argtypes = [ctypes.c_void_p, ctypes.c_int64]
L.gprx_dev_bs_trace.restype = ctypes.c_int64
ctx = gpr_amd.Context(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else C3["n"]
X, Y = make_data(n, C3["d"], C3["m"])
M = gpr_amd.Model(ctx, np.float64)
M.set_data(X, Y)
M.set_kernel(C3["kernel"])
M.set_noise(C3["sigma"])
M.fit()
info = M.fit()
nb = (n + 127) // 128
tr = np.zeros((nb, 4), np.int64)
k = L.gprx_dev_bs_trace(tr.ctypes.data, nb)
t = (tr - tr[:, 0].min()) / 100.0  # us
pub = t[:, 3]
step = pub[:-1] - pub[1:]           # alpha_k published minus alpha_{k+1} published
crit = t[:-1, 3] - t[:-1, 2]        # alpha_{k+1} seen -> alpha_k published
seen_lag = t[:-1, 2] - pub[1:]      # alpha_{k+1} published -> seen by block k
late = t[:-1, 1] - pub[1:]          # non-critical done relative to alpha_{k+1} published
print(json.dumps({"blocks": int(k), "ms_solve": info.ms_solve, "span_us": float(pub.max() - t[:, 0].min()),
                  "step_us_mean": float(step.mean()), "step_us_p90": float(np.percentile(step, 90)),
                  "crit_us_mean": float(crit.mean()), "seen_lag_us_mean": float(seen_lag.mean()),
                  "noncrit_late_us_mean": float(late.mean()), "noncrit_late_frac": float((late > 0).mean()),
                  "first_start_to_last_start_us": float(t[:, 0].max() - t[:, 0].min())}, indent=1))
