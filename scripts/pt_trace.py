"""Timeline of one tile-dataflow factorisation (GPRX_PT_TRACE): per-type task durations,
waits, worker utilisation and the DIAGX chain."""
import ctypes, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("GPRX_PT_TRACE", "1")
import numpy as np
import gpr_amd
from gpr_amd.gprx import lib

L = lib()
L.gprx_dev_bench.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64,
                             ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_double)]
L.gprx_dev_pt_trace.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
L.gprx_dev_pt_trace.restype = ctypes.c_int64
ctx = gpr_amd.Context(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
ms = ctypes.c_double()
if os.environ.get("PT_TRACE_FIT"):  # the C3 fit (fused covariance build) instead of a bare factorisation
    from gpr_amd.synth import C3, make_data
    X, Y = make_data(n, C3["d"], C3["m"])
    M = gpr_amd.Model(ctx, np.float64)
    M.set_data(X, Y)
    M.set_kernel(C3["kernel"])
    M.set_noise(C3["sigma"])
    M.fit()
    info = M.fit()
    ms.value = info.ms_factor
    n = ((n + 127) // 128) * 128
else:
    dt = int(os.environ.get("PT_TRACE_DTYPE", "1"))  # 1: f64, 0: f32 (gprx_dtype)
    assert L.gprx_dev_bench(ctx.h, dt, 9, n, 0, 0, 2, ctypes.byref(ms)) == 0
MAX = 400000
tasks = np.zeros((MAX, 4), np.int32)
times = np.zeros((MAX, 4), np.int64)
k = L.gprx_dev_pt_trace(tasks.ctypes.data, times.ctypes.data, MAX)
ntask = int(((k - 1) // 1))
# the last nc rows of `times` are DIAGX phase stamps {trsm done, published, syrk done, diag done}
nc = n // 128
nt = k - 7 * nc                         # rows: tickets, DIAGX phases, diag_factor, TPART / split stamps
dph = times[nt:nt + nc].copy()
dprof = times[nt + nc:nt + 2 * nc].copy()  # diag_factor {load, pivot phases, update phases} ticks
xtp = times[nt + 2 * nc:nt + 6 * nc].reshape(nc, 4, 4).copy()  # TPART(k, c) stamps
xdg = times[nt + 6 * nc:nt + 7 * nc].copy()                   # split DIAGX(k) stamps
tasks, times = tasks[:nt], times[:nt]
out = os.environ.get("PT_TRACE_OUT")
if out:
    np.savez_compressed(out, tasks=tasks, times=times)
t0 = times[:, 0].min()
tk = (times[:, :3] - t0) / 100.0  # us
span = tk[:, 2].max()
typ = tasks[:, 0] & 0xff
nb = tasks[:, 0] >> 8
ex = tk[:, 2] - tk[:, 1]
wt = tk[:, 1] - tk[:, 0]
P = len(np.unique(times[:, 3] & 0xffff))
cyc = times[:, 3] >> 16
dur_ticks = times[:, 2] - times[:, 1]
okc = dur_ticks > 500
clock_ghz = float(np.median(cyc[okc] / dur_ticks[okc]) * 0.1)
res = {"clock_ghz_median": clock_ghz, "n": n, "ms_devbench": ms.value, "span_us": span, "tasks": int(k), "workers": P,
       "busy_frac": float(ex.sum() / (span * P)), "wait_frac": float(wt.sum() / (span * P))}
names = {0: "DIAGX", 1: "TRSM", 2: "UPD", 3: "BUILD", 4: "TPART", 5: "UPD2"}
for t in (0, 1, 2, 3, 4, 5):
    for b in sorted(set(nb[typ == t])):
        m = (typ == t) & (nb == b)
        diag = (tasks[:, 1] == tasks[:, 2])
        key = f"{names[t]}{'' if t not in (2, 5) else '_nb' + str(b)}"
        if t == 4:  # the split diagonal step's parts, by column block c
            for c in range(4):
                mc = m & (tasks[:, 2] == c)
                if mc.any():
                    res[f"TPART_c{c}"] = {"count": int(mc.sum()), "exec_us_mean": float(ex[mc].mean()),
                                          "wait_us_mean": float(wt[mc].mean())}
            continue
        res[key] = {"count": int(m.sum()), "exec_us_mean": float(ex[m].mean()), "exec_us_p90": float(np.percentile(ex[m], 90)),
                    "wait_us_mean": float(wt[m].mean())}
        if t == 2:
            md = m & diag
            if md.any():
                res[key]["diagtile_exec_us_mean"] = float(ex[md].mean())
# worker time per task type, in ms of the whole chip (sum of exec / workers)
res["chip_ms_by_type"] = {names[t]: round(float(ex[typ == t].sum() / P / 1e3), 3) for t in (0, 1, 2, 3, 4, 5)}
res["chip_ms_wait"] = round(float(wt.sum() / P / 1e3), 3)
res["chip_ms_idle"] = round(float(span / 1e3 - (ex.sum() + wt.sum()) / P / 1e3), 3)
res["upd_panels"] = int(nb[typ == 2].sum())
res["upd2_panels"] = int(nb[typ == 5].sum())  # (each covers two tiles)
# DIAGX chain
d = np.where(typ == 0)[0]
order = np.argsort(tasks[d, 1])
d = d[order]
st = tk[d, 1]
en = tk[d, 2]
res["diagx_exec_mean_us"] = float((en - st).mean())
gaps = st[1:] - en[:-1]
res["diagx_gap_mean_us"] = float(gaps.mean())
res["diagx_chain_first_last"] = [float(st[0]), float(en[-1])]
# the chain's period: DIAGX(k) end - DIAGX(k-1) end (the split step's parts included)
per = en[1:] - en[:-1]
res["chain_period_us"] = {"mean": float(per.mean()), "median": float(np.median(per)),
                          "last16_mean": float(per[-16:].mean())}
# time profile: busy workers per 1 ms window
bins = np.arange(0, span + 1000, 1000)
busy = []
for a in bins[:-1]:
    b = a + 1000
    ov = np.clip(np.minimum(tk[:, 2], b) - np.maximum(tk[:, 1], a), 0, None)
    busy.append(round(float(ov.sum() / 1000 / P), 2))
res["busy_per_ms"] = busy
# late chain: k -> diag exec and gap for last 16
dv = dph[1:]
res["diagx_phase_us"] = {"trsm_tile": float(np.mean((dv[:, 0] - (times[d[1:], 1])) / 100.0)),
                         "publish": float(np.mean((dv[:, 1] - dv[:, 0]) / 100.0)),
                         "syrk_tile": float(np.mean((dv[:, 2] - dv[:, 1]) / 100.0)),
                         "diag_factor": float(np.mean((dv[:, 3] - dv[:, 2]) / 100.0)),
                         "final_publish": float(np.mean((times[d[1:], 2] - dv[:, 3]) / 100.0))}
res["diag_factor_us"] = {"load": float(dprof[:, 0].mean() / 100), "pivot_solve": float(dprof[:, 1].mean() / 100),
                         "update": float(dprof[:, 2].mean() / 100)}
# the split step: per k >= 1, microseconds after Linv_{k-1} was published (DIAGX(k-1) done)
if (xtp[1:, :, 0] > 0).all():
    t_lin = tk[d[:-1], 2] * 100.0 + t0  # DIAGX(k-1) published, ticks
    rel = lambda a: (a - t_lin[:, None]) / 100.0
    ph = {}
    for c in range(4):
        s_ = xtp[1:, c, :]
        ph[f"c{c}"] = {"linv_seen": float(np.median(rel(s_[:, :1]))), "t_done": float(np.median(rel(s_[:, 1:2]))),
                       "t_stored": float(np.median(rel(s_[:, 2:3]))), "s_quarter_done": float(np.median(rel(s_[:, 3:4])))}
        tpi = np.where((typ == 4) & (tasks[:, 2] == c))[0]
        tpi = tpi[np.argsort(tasks[tpi, 1])]
        ph[f"c{c}"]["published"] = float(np.median((tk[tpi, 2] * 100.0 + t0 - t_lin) / 100.0))
    dgs = xdg[1:]
    ph["diagx"] = {"start": float(np.median((tk[d[1:], 1] * 100.0 + t0 - t_lin) / 100.0)),
                   "quarters_seen": float(np.median(rel(dgs[:, 2:3]))), "s_done": float(np.median(rel(dgs[:, 3:4]))),
                   "end": float(np.median((tk[d[1:], 2] * 100.0 + t0 - t_lin) / 100.0))}
    res["split_step_us"] = ph
res["diagx_last16"] = [[round(float(e - s_), 1), round(float(g), 1)] for s_, e, g in zip(st[-16:], en[-16:], np.r_[gaps, 0][-16:])]
print(json.dumps(res, indent=1))
