#!/usr/bin/env python3
"""bench.py — GP fits/sec on the BASELINE.json headline configuration.

Workload (BASELINE.json configs[2], the config the metric "GP fits/sec + predict pts/sec,
N=16384 d=32 fp64" is quoted on): N=16384 training points, d=32, m=1, fp64,
SumKernel(GaussianKernel(2,0.15), PeriodicKernel(0.1,pi,1)), noise sigma=1.0, synthetic
SplitMix64 data (gpr_amd/synth.py).  One step = one full GP fit = covariance build +
Cholesky factorisation + regression-vector solve (the reference's
GaussianProcess<double>::Initialize, lib/GaussianProcess.cpp:118-130), inputs resident in
HBM before the timed region.

Multi-GPU: launched by torch.distributed.run, one process per GPU.  The headline (--mode
dist, the default for N > 1) is ONE fit per step whose matrix is sharded over the ranks:
row blocks dealt in cyclic groups (each GPU stores only the lower tiles of its own row blocks,
~N^2/(2g), and builds only those), each rank runs the persistent tile-dataflow factorisation on
its rows, and the exchange is device-initiated: a finished tile is stored by the task that
produced it straight into the windows of the ranks that read it (IPC-mapped over xGMI), the
diagonal-block inverses likewise into every rank (gpr_amd/csrc/gprx_dist.cpp; strong scaling:
value = fits/s of the job).  The same run also measures --mode replicas (every rank fits its
own GP, weak scaling) and reports it under "replicas"; `--mode replicas` makes that the
headline.  Predict is query-sharded over the ranks (X and alpha replicated).

The other BASELINE.json configurations are measured in the same run ("configs" in the JSON
line, --configs 0 skips them), each with its own dominant-kernel roofline and a labelled CPU
baseline: C2 (N=4096 d=16 Gaussian fp64, replicas), C4 (N=32768 d=32 RationalQuadratic fp32 with
the fp64 refinement; sharded over the ranks for N > 1, its BASELINE form), C5 (sparse GP M=2048
inducing, N=1e6 d=64 fp64, dense rows sharded over the ranks).

Prints ONE JSON line on rank 0 (plus human-readable detail on stderr).
"""
import argparse
import csv
import glob
import json
import os
import re
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP64_TFLOPS = 78.6   # MI355X dense fp64 (vector = matrix), MI355X_MICROARCH.md / SURVEY.md §8(d)
PEAK_FP32_TFLOPS = 157.3  # MI355X dense fp32 matrix
PEAK_HBM_GBS = 8000.0     # HBM3E spec
# the measured parts of one bench run; `--legs` selects a subset (one leg per profiled process)
LEGS = ("c3", "predict", "variance", "lml", "build", "c2", "c4", "c5")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def fit_roofline_ms(n, d, m, gpus=1):
    """T_roof = B_build/BW + F_potrf/(peak*g) + B_solve/BW (comm excluded)."""
    b_build = 8.0 * (n * d + n * (n + 1) / 2)
    f_potrf = n ** 3 / 3.0
    b_solve = 2 * 8.0 * n * (n + 1) / 2 * m
    return 1e3 * (b_build / (PEAK_HBM_GBS * 1e9) + f_potrf / (PEAK_FP64_TFLOPS * 1e12 * gpus)
                  + b_solve / (PEAK_HBM_GBS * 1e9))


def host_info():
    """The CPU the baselines ran on (nproc, CPU model and RAM beside the
    result): /proc/cpuinfo's model name, /proc/meminfo's MemTotal, the CPUs this process may use."""
    model, ram = None, None
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), None)
        with open("/proc/meminfo") as f:
            kb = next((int(ln.split()[1]) for ln in f if ln.startswith("MemTotal")), None)
        ram = round(kb / 2 ** 20, 1) if kb else None
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = os.cpu_count()
    return {"cpu_model": model, "ram_gib": ram, "cpus_usable": usable, "cpus_machine": os.cpu_count()}


def _cpu_warmup(O, cfg):
    """One untimed small call (thread pool start, MKL initialisation, page faults of the code)
    before a timed CPU leg, so no leg's first sample carries the cold start."""
    from gpr_amd.synth import make_data
    X, Y = make_data(512, cfg["d"], cfg["m"])
    O.fit(cfg["kernel"], X, Y, cfg["sigma"], np.float64, want_core=False)


def cpu_baseline(cfg, n_cpu):
    """The CPU restatement of the reference's fit (oracle/: kernel pair loop + LAPACK
    dgetrf+dgetri in fp64 + C*Y), timed on this host's cores: one fit at n_cpu after a warm-up."""
    from oracle import oracle as O
    from gpr_amd.synth import make_data
    _cpu_warmup(O, cfg)
    X, Y = make_data(n_cpu, cfg["d"], cfg["m"])
    t0 = time.perf_counter()
    O.fit(cfg["kernel"], X, Y, cfg["sigma"], np.float64, want_core=False)
    dt = time.perf_counter() - t0
    scale = (n_cpu / cfg["n"]) ** 3  # fits/s at the bench N (LU inverse is 2N^3)
    return dict({
        "value": (1.0 / dt) * scale,
        "unit": "fits/s",
        "cores": O.num_threads(),
        "kind": "port",
        "sample": (f"1 fit at N={n_cpu} (d={cfg['d']}, same kernel) in {dt:.2f} s after a warm-up, LAPACK={O.lapack_name()}"
                   + ("" if n_cpu == cfg["n"] else f", cubic-scaled to N={cfg['n']}")),
    }, **host_info())


def cpu_lml_baseline(cfg, ns, t_gpu_ms=None):
    """The CPU restatement of the reference's log-marginal likelihood + gradient
    (GaussianLogLikelihood::GetValueAndParameterDerivatives, include/Likelihood.h:231-285:
    K, the LU inverse C in fp64, the long-double determinant of lib/GaussianProcess.cpp:513-528,
    the P derivative matrices and tr((alpha alpha^T - C) dK_p)) timed at the sizes `ns` on this
    host's cores and EXTRAPOLATED to the bench N by the cubic t(n) = a n^3 + b n^2 + c through
    the measured points (a full run at N = 16384 is dominated by the
    long-double determinant, est. >= 30 min)."""
    from oracle import oracle as O
    from gpr_amd.synth import make_data
    X, Y = make_data(512, cfg["d"], cfg["m"])  # (untimed warm-up: thread pool, MKL, code pages)
    O.lml(cfg["kernel"], X, Y, cfg["sigma"], np.float64, with_grad=True)
    ts = []
    for n_ in ns:
        X, Y = make_data(n_, cfg["d"], cfg["m"])
        t0 = time.perf_counter()
        O.lml(cfg["kernel"], X, Y, cfg["sigma"], np.float64, with_grad=True)
        ts.append(time.perf_counter() - t0)
    n = cfg["n"]
    nn = np.array(ns, dtype=np.float64)
    tt = np.array(ts)
    pure = ts[-1] * (n / ns[-1]) ** 3
    fit = None
    if len(ns) >= 2:
        # t(n) = a n^3 + b n^2 by least squares RELATIVE to each point (two terms: with three
        # points a third would fit them exactly and say nothing about the fit's quality); the
        # residual is the largest relative miss at the measured points
        A = np.stack([nn ** 3, nn ** 2], axis=1) / tt[:, None]
        coef = np.linalg.lstsq(A, np.ones_like(tt), rcond=None)[0]
        pred = coef[0] * nn ** 3 + coef[1] * nn ** 2
        fit = {"a_n3": float(coef[0]), "b_n2": float(coef[1]),
               "max_rel_residual": float(np.max(np.abs(pred - tt) / tt)),
               "t_extrapolated_s": float(coef[0] * n ** 3 + coef[1] * n ** 2)}
    if fit is not None and fit["a_n3"] > 0 and fit["t_extrapolated_s"] >= ts[-1] * (n / ns[-1]) ** 2:
        t_n, how = fit["t_extrapolated_s"], "least-squares a n^3 + b n^2 through the points (relative)"
    else:
        t_n, how = pure, "pure cubic from the largest point"
    return dict({
        "value": 1.0 / t_n,
        "unit": "LML+gradient evaluations/s",
        "ms_extrapolated": 1e3 * t_n,
        "cores": O.num_threads(),
        "kind": "port",
        "extrapolated": True,
        "points": {str(a): b for a, b in zip(ns, ts)},
        "fit": fit,
        "ms_pure_cubic_from_largest": 1e3 * pure,
        "sample": (f"oracle LML + gradient (LU inverse via LAPACK {O.lapack_name()}, long-double determinant, "
                   f"P={5} derivative traces) after a warm-up, measured at N={list(ns)}: "
                   + ", ".join(f"{t:.2f} s" for t in ts) + f"; EXTRAPOLATED to N={n} by {how}"),
        "gpu_over_cpu": (t_n * 1e3 / t_gpu_ms) if t_gpu_ms else None,
    }, **host_info())


def cpu_predict_baseline(cfg, X, alpha, q_cpu):
    """The reference's Predict (lib/GaussianProcess.cpp:54-61: one kernel vector k(x, X) and a
    dot with alpha per point, apps/GaussianProcessPredict.cpp:185-193 loops over the points)
    restated (oracle predict, OpenMP over the points) and timed on this host's cores for q_cpu
    queries against the same N-sample model."""
    from oracle import oracle as O
    from gpr_amd.synth import make_queries
    Xq = make_queries(q_cpu, cfg["d"])
    O.predict(cfg["kernel"], X, alpha, Xq[:64])  # (thread pool, pages)
    t0 = time.perf_counter()
    O.predict(cfg["kernel"], X, alpha, Xq)
    dt = time.perf_counter() - t0
    return dict({"value": q_cpu / dt, "unit": "pts/s", "cores": O.num_threads(), "kind": "port",
                 "sample": f"{q_cpu} query points against the N={cfg['n']} d={cfg['d']} model (oracle per-point "
                           f"predict, OpenMP over the points) in {dt:.2f} s after a warm-up"}, **host_info())


def _short(name):
    """Kernel name without `void`, namespaces and the argument list (as scripts/pmc_traffic.py)."""
    m = re.match(r"(?:void )?(?:[A-Za-z_0-9]+::)*([A-Za-z_0-9]+<[^()]*>|[A-Za-z_0-9]+)", name)
    return m.group(1) if m else name


def _tagged(pattern):
    """Committed profile summaries matching profiles/<pattern>, oldest first: tags r<round><a..z,
    aa..az ...> order by round, then by the tag's length and letters (r03ak after r03t)."""
    def order(path):
        m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")
    return sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)), key=order)


def traffic_from_profile(leg="c3", kernels=("potrf_tiles_kernel<double, false>",)):
    """HBM bytes per launch of a leg's dominant kernel from the newest committed rocprofv3 PMC
    passes of that leg (profiles/<tag>_<leg>_pmc_traffic.json, scripts/pmc_traffic.py; for the
    C3 fit also the older leg-less profiles/<tag>_pmc_traffic.json).  L2-fabric bytes:
    FETCH_SIZE x 2 -- the gfx950 correction for 16-B-per-lane streaming reads, which is how the
    tile kernel reads all of its operands (MI355X_MICROARCH.md §HBM) -- + WRITE_SIZE, averaged
    over launches; Infinity-Cache hits are included, so this bounds HBM bytes from above."""
    files = _tagged(f"*_{leg}_pmc_traffic.json")
    if leg == "c3" and not files:
        files = [p for p in _tagged("*_pmc_traffic.json") if re.match(r"r\d+[a-z]*_pmc_traffic", os.path.basename(p))]
    for path in reversed(files):
        try:
            with open(path) as f:
                ks = json.load(f)["kernels"]
            k = next((ks[n] for n in kernels if n in ks), None)
        except Exception:
            continue
        if k is not None:
            return {"bytes_per_launch": k["hbm_bytes_per_launch"], "source": os.path.basename(path)}
    return None


def rocprof_from_profile(leg, kernels, inrun_us=None):
    """The average launch duration of a leg's dominant kernel in the newest committed
    `rocprofv3 --kernel-trace --stats` summary of that leg (profiles/<tag>_<leg>_kernel_stats.csv,
    one profiled bench.py process per leg: scripts/gpu.sh profile), beside this run's in-run
    HIP-event average, so every roofline in the line can be checked against a profile."""
    for path in reversed(_tagged(f"*_{leg}_kernel_stats.csv")):
        try:
            with open(path) as f:
                rows = [r for r in csv.DictReader(f) if _short(r["Name"]) in kernels]
        except Exception:
            continue
        if rows:
            r = max(rows, key=lambda r: float(r["TotalDurationNs"]))
            avg = float(r["AverageNs"]) / 1e3
            return {"avg_us": avg, "calls": int(r["Calls"]), "kernel": _short(r["Name"]),
                    "source": os.path.basename(path),
                    "inrun_over_rocprof": (inrun_us / avg) if inrun_us else None}
    return None


def rocprof_table(leg, min_percent=1.0):
    """Every kernel above `min_percent` of the device time in the newest committed kernel-stats
    summary of a leg (the LML's several launches)."""
    files = _tagged(f"*_{leg}_kernel_stats.csv")
    if not files:
        return None
    with open(files[-1]) as f:
        rows = [r for r in csv.DictReader(f) if float(r["Percentage"]) >= min_percent]
    return {"source": os.path.basename(files[-1]),
            "kernels": {_short(r["Name"]): {"avg_us": float(r["AverageNs"]) / 1e3, "calls": int(r["Calls"])}
                        for r in rows}}


def mfma_from_profile(leg, kernels):
    """MFMA-busy fraction of a leg's dominant kernel from the newest committed PMC pass
    (profiles/<tag>_<leg>_pmc_mfma.json, scripts/pmc_mfma.py), averaged over its launches."""
    for path in reversed(_tagged(f"*_{leg}_pmc_mfma.json")):
        try:
            with open(path) as f:
                ks = json.load(f)["kernels"]
            v = next((ks[n] for n in kernels if n in ks), None)
        except Exception:
            continue
        if v:
            return {"mfma_busy_frac": float(np.mean([x["mfma_busy_frac"] for x in v])),
                    "clock_ghz": float(np.mean([x["clock_ghz"] for x in v])), "launches": len(v),
                    "source": os.path.basename(path)}
    return None


def predict_pmc_from_profile():
    """The predict kernel's issue split from the newest committed PMC passes
    (profiles/<tag>_predict_pmc.json, scripts/pmc_generic.py): MFMA busy and VALU issue as
    fractions of the SIMD-cycles, the wait split of the wave-cycles, LDS bank conflicts."""
    for path in reversed(_tagged("*_predict_pmc.json")):
        try:
            with open(path) as f:
                ks = json.load(f)["kernels"]
            k = next((v for n, v in ks.items() if n.startswith("predict_mma_kernel")), None)
        except Exception:
            continue
        if k:
            keys = ("mfma_busy_frac", "valu_active_frac", "wait_inst_frac", "wait_any_frac", "active_any_frac",
                    "lds_conflict_frac", "clock_ghz", "dur_ms_mean")
            return dict({x: k.get(x) for x in keys}, source=os.path.basename(path))
    return None


def make_dist_context(gpr_amd, group, rank, world, local_rank, shared):
    """The multi-process context of the sharded fit: an RCCL communicator over the GPUs
    (gprx_ctx_create_dist, nonblocking initialisation with a deadline), or, when any rank's
    RCCL initialisation fails or times out, every rank falls back to the peer context over the
    host group's all-gather (gprx_ctx_create_peer: the same device-initiated exchange, host
    collectives over the sockets instead of RCCL).  The ranks agree on the choice.  Returns
    (context, transport, error-or-None).  GPRX_DIST_SHARED_GPU (one GPU for every rank, which
    RCCL refuses) goes to the peer context directly."""
    if group is None:  # --force-dist at N = 1: a one-rank RCCL communicator
        return gpr_amd.Context(local_rank, dist=(0, 1, gpr_amd.unique_id())), "rccl", None
    # (a shared-GPU rehearsal tries RCCL only under GPRX_RCCL_FAIL, which fails it on purpose:
    # the fallback below, rehearsed on one GPU)
    if shared and os.environ.get("GPRX_RCCL_FAIL", "0") == "0":
        return gpr_amd.Context(0, peer=(rank, world, group.allgather_fn())), "peer (shared GPU)", None
    err = None
    ctx = None
    try:
        uid = group.broadcast(gpr_amd.unique_id() if rank == 0 else None)
        ctx = gpr_amd.Context(local_rank, dist=(rank, world, uid))
    except Exception as e:
        err = f"rank {rank}: RCCL context: {e!r}"
        log(err)
    errs = [e.decode() for e in group.allgather((err or "").encode()) if e]
    if not errs:
        return ctx, "rccl", None
    if ctx is not None:
        ctx.close()  # (ncclCommAbort: local, never waits on the ranks that failed)
    ctx = gpr_amd.Context(local_rank, peer=(rank, world, group.allgather_fn()))
    return ctx, "peer (fallback: RCCL initialisation failed)", "; ".join(errs)


def chain_from_trace(path):
    """The diagonal chain as this rank saw it, from a GPRX_DIST_TRACE_FILE dump of one sharded
    fit (gprx_dist.cpp: int32 ntasks, rank, g, nc; int4 per ticket; 4 int64 per ticket: taken,
    inputs ready, published, workgroup, 100 MHz ticks).  DIAGX(k) is ticket type 0 with k in
    field 1.  chain_step_us: median of publish(k) - publish(k-1) over the consecutive steps this
    rank owns both of (one rank's clock); exec_us: DIAGX's mean duration."""
    raw = open(path, "rb").read()
    nt, r, g, nc = (int(v) for v in np.frombuffer(raw[:16], np.int32))
    tasks = np.frombuffer(raw[16:16 + 16 * nt], np.int32).reshape(nt, 4)
    times = np.frombuffer(raw[16 + 16 * nt:16 + 48 * nt], np.int64).reshape(nt, 4)
    sel = (tasks[:, 0] & 0xff) == 0
    ks, pub, ready = tasks[sel, 1], times[sel, 2], times[sel, 1]
    o = np.argsort(ks)
    ks, pub, ready = ks[o], pub[o], ready[o]
    cons = np.where(np.diff(ks) == 1)[0]
    steps = (pub[cons + 1] - pub[cons]) / 100.0
    span = (times[:, 2].max() - times[:, 0].min()) / 100.0
    return {"diag_steps_owned": int(len(ks)), "chain_step_us_median": float(np.median(steps)) if len(steps) else None,
            "chain_step_us_mean": float(np.mean(steps)) if len(steps) else None, "consecutive_pairs": int(len(steps)),
            "diagx_exec_us_mean": float(np.mean((pub - ready) / 100.0)) if len(ks) else None,
            "launch_span_us": float(span), "tickets": int(nt)}


def dist_rank_record(ctx, model, transport):
    """This rank's identity and exchange figures for the N > 1 line: the device (ordinal and PCI
    address), the transport, the RCCL communicator's own rank count, the Linv / tile pushes of
    one fit and their bytes (from the schedule, gprx_dev_dist_info), and the chain step measured
    on a traced fit."""
    rec = dict(ctx.info())
    rec["transport_bench"] = transport
    di = model.dist_info()
    rec.update({k: di[k] for k in ("push_linv", "push_tiles", "push_bytes", "gb", "ww", "P", "est_us",
                                   "bytes_rank", "bytes_storage")})
    base = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"gprx_chain_{os.getpid()}")
    os.environ["GPRX_DIST_TRACE_FILE"] = base
    try:
        info = model.fit(gpr_amd_fit_flag())
        rec["traced_fit_ms_factor"] = float(info.ms_factor)
    finally:
        del os.environ["GPRX_DIST_TRACE_FILE"]
    path = f"{base}.r{rec['rank']}"
    try:
        rec.update(chain_from_trace(path))
    finally:
        for f in glob.glob(base + ".r*"):
            os.remove(f)
    return rec


def gpr_amd_fit_flag():
    from gpr_amd.gprx import FIT_DISTRIBUTED
    return FIT_DISTRIBUTED


class _Skip(Exception):
    """A leg left out by --legs."""


def run_configs(args, world, rank, local_rank, dctx, max_over_ranks, barrier_sync, want):
    """BASELINE.json configs[1], [3], [4] (C2, C4, C5), each timed like the headline (warmup,
    then K steps between barriers, max over ranks) with the dominant kernel's roofline from its
    HIP-event device time, and (rank 0, N = 1) a labelled CPU baseline on a bounded sample."""
    import gpr_amd
    from gpr_amd.synth import C2, C4, make_data
    from gpr_amd.gprx import FIT_DISTRIBUTED
    out = {}

    def fit_leg(cfg, ctx, flags, dtype, steps):
        X, Y = make_data(cfg["n"], cfg["d"], cfg["m"])
        M = gpr_amd.Model(ctx, dtype)
        M.set_data(X.astype(dtype), Y.astype(dtype))
        M.set_kernel(cfg["kernel"])
        M.set_noise(cfg["sigma"])
        for _ in range(max(1, args.warmup)):
            M.fit(flags)
        ctx.set_stats(True)
        barrier_sync()
        t0 = time.perf_counter()
        infos = [M.fit(flags) for _ in range(steps)]
        barrier_sync()
        el = max_over_ranks(time.perf_counter() - t0)
        st = ctx.stats()
        ctx.set_stats(False)
        dinfo = M.dist_info() if flags & FIT_DISTRIBUTED else None
        M.close()
        return el, infos, st, dinfo

    # ---- C2: N=4096 d=16 GaussianKernel fp64 (replicas: every rank fits its own) -----------------
    try:
        if not want("c2"):
            raise _Skip
        n, m = C2["n"], C2["m"]
        ctx = gpr_amd.Context(local_rank)
        el, infos, st, _ = fit_leg(C2, ctx, 0, np.float64, max(args.steps, 10))
        ctx.close()
        steps = max(args.steps, 10)
        fac = st.get("potrf_tiles", {"ms": 0, "launches": 0})
        t_k = max_over_ranks(fac["ms"] / fac["launches"]) if fac["launches"] else None
        alg = n ** 3 / 3.0 + m * float(n) ** 2
        c2 = {"workload": "C2: GP fit N=4096 d=16 m=1 GaussianKernel(1,1) sigma=0.1 fp64 (BASELINE.json configs[1])",
              "metric": "GP fits/sec", "value": world * steps / el, "unit": "fits/s", "ms_per_step": 1e3 * el / steps,
              "scaling": "weak" if world > 1 else None, "dtype": "f64",
              "roofline": {"bound": "mfma", "kernel": "potrf_tiles_kernel<double, false> (fused build + Cholesky)",
                           "achieved": alg / (t_k * 1e-3) / 1e12 if t_k else None, "peak": PEAK_FP64_TFLOPS,
                           "unit": "TFLOP/s", "frac": alg / (t_k * 1e-3) / 1e12 / PEAK_FP64_TFLOPS if t_k else None,
                           "avg_launch_us": 1e3 * t_k if t_k else None, "algorithmic_flops_per_launch": alg,
                           "note": "latency-bound: N/128 = 32 serial diagonal steps"}}
        c2["roofline"]["rocprof"] = rocprof_from_profile("c2", ("potrf_tiles_kernel<double, false>",),
                                                         c2["roofline"]["avg_launch_us"])
        if rank == 0 and world == 1 and args.cpu_n > 0:
            from oracle import oracle as O
            _cpu_warmup(O, C2)
            X, Y = make_data(n, C2["d"], m)
            dts = []
            for _ in range(3):  # the median of three full fits (one cold sample swung 7x between boxes)
                t0 = time.perf_counter()
                O.fit(C2["kernel"], X, Y, C2["sigma"], np.float64, want_core=False)
                dts.append(time.perf_counter() - t0)
            dt = float(np.median(dts))
            c2["cpu_baseline"] = dict({"value": 1.0 / dt, "unit": "fits/s", "cores": O.num_threads(), "kind": "port",
                                       "samples_s": dts,
                                       "sample": f"median of 3 full fits at N={n} after a warm-up (oracle: kernel loop + "
                                                 f"LAPACK {O.lapack_name()} getrf+getri in fp64 + C Y): {dt:.3f} s"},
                                      **host_info())
        out["C2"] = c2
    except _Skip:
        pass
    except Exception as e:
        out["C2"] = {"error": repr(e)}
    # ---- C4: N=32768 d=32 RationalQuadratic fp32 (sharded for N > 1, its BASELINE form) ----------
    try:
        if not want("c4"):
            raise _Skip
        n, m = C4["n"], C4["m"]
        steps = max(3, min(args.steps, 5))
        if world > 1 and dctx is not None:
            el, infos, st, dinfo = fit_leg(C4, dctx, FIT_DISTRIBUTED, np.float32, steps)
            t_k = max_over_ranks(float(np.mean([i.ms_factor for i in infos])))
            kname = "potrf_tiles_kernel<float, true> (one per rank, sharded)"
            peak = PEAK_FP32_TFLOPS * world
        else:
            ctx = gpr_amd.Context(local_rank)
            el, infos, st, dinfo = fit_leg(C4, ctx, 0, np.float32, steps)
            ctx.close()
            fac = st.get("potrf_tiles", {"ms": 0, "launches": 0})
            t_k = fac["ms"] / fac["launches"] if fac["launches"] else None
            kname = "potrf_tiles_kernel<float, false> (Cholesky + forward solve)"
            peak = PEAK_FP32_TFLOPS
        alg = n ** 3 / 3.0 + m * float(n) ** 2
        c4 = {"workload": "C4: GP fit N=32768 d=32 m=1 RationalQuadraticKernel(1,0.3,1) sigma=1.0 fp32, alpha refined "
                          "in fp64 (BASELINE.json configs[3])",
              "metric": "GP fits/sec", "value": steps / el, "unit": "fits/s", "ms_per_step": 1e3 * el / steps,
              "n_gpus": world, "scaling": "strong" if world > 1 else None, "dtype": "f32 (factor) + f64 (refinement)",
              "refine_steps": int(infos[-1].refine_steps), "refine_delta": float(infos[-1].refine_delta),
              "ms_refine": float(np.mean([i.ms_refine for i in infos])),
              "roofline": {"bound": "mfma", "kernel": kname,
                           "achieved": alg / (t_k * 1e-3) / 1e12 if t_k else None, "peak": peak, "unit": "TFLOP/s",
                           "frac": alg / (t_k * 1e-3) / 1e12 / peak if t_k else None,
                           "avg_launch_us": 1e3 * t_k if t_k else None, "algorithmic_flops_per_launch": alg},
              "dist": dinfo}
        if world == 1:
            c4["roofline"]["rocprof"] = rocprof_from_profile("c4", ("potrf_tiles_kernel<float, false>",),
                                                             c4["roofline"]["avg_launch_us"])
            c4["roofline"]["mfma_busy"] = mfma_from_profile("c4", ("potrf_tiles_kernel<float, false>",))
        if rank == 0 and world == 1 and args.cpu_n > 0:
            from oracle import oracle as O
            _cpu_warmup(O, C4)
            ns = 8192
            X, Y = make_data(ns, C4["d"], m)
            t0 = time.perf_counter()
            O.fit(C4["kernel"], X.astype(np.float32), Y.astype(np.float32), C4["sigma"], np.float32, want_core=False)
            dt = time.perf_counter() - t0
            c4["cpu_baseline"] = dict({"value": 1.0 / (dt * (n / ns) ** 3), "unit": "fits/s", "cores": O.num_threads(),
                                       "kind": "port", "extrapolated": True,
                                       "sample": f"1 fit at N={ns} after a warm-up (oracle fp32 path: K in fp32 cast to "
                                                 f"double, LAPACK {O.lapack_name()} getrf+getri) in {dt:.2f} s, "
                                                 f"EXTRAPOLATED cubically to N={n}"}, **host_info())
        out["C4"] = c4
    except _Skip:
        pass
    except Exception as e:
        out["C4"] = {"error": repr(e)}
    # ---- C5: sparse GP M=2048, N=1e6, d=64 fp64 (dense rows sharded over the ranks) ------------
    try:
        if not want("c5"):
            raise _Skip
        n, M_, d = 1_000_000, 2048, 64
        ks, sig, jit = "GaussianKernel(3,1,)", 0.1, 1e-4
        X, Y = make_data(n, d, 1)
        Xm = X[:: n // M_][:M_].copy()
        rows = np.array_split(np.arange(n), world)[rank]
        Xl, Yl = X[rows].copy(), Y[rows].copy()
        del X, Y
        ctx = dctx if (world > 1 and dctx is not None) else gpr_amd.Context(local_rank)
        # the rank's rows resident in HBM before the timed region (the value's rule); the
        # PCIe-inclusive rate from host arrays is reported beside it
        # (the library's own device buffers: torch's bundled HIP runtime cannot allocate once
        # this library owns the device, so torch CUDA tensors are not an option here)
        resident = False
        try:
            Xr, Yr = ctx.device_array(Xl), ctx.device_array(Yl)
            resident = True
        except Exception as e:  # (the host arrays then, labelled)
            log("C5: device-resident inputs unavailable:", e)
        Xin, Yin = (Xr, Yr) if resident else (Xl, Yl)
        # the M x M results stay in HBM as well (the dense fit's alpha does: the model keeps it);
        # the host-output rate is the PCIe-inclusive figure below
        outs = None
        if resident:
            outs = tuple(gpr_amd.DeviceArray.empty(ctx, shp) for shp in ((M_, M_), (M_, 1), (M_, M_)))
        ctx.sparse_fit(ks, Xin, Yin, Xm, sig, jit, out=outs)
        steps = max(3, min(args.steps, 5))
        barrier_sync()
        tp0 = time.perf_counter()
        ctx.sparse_fit(ks, Xl, Yl, Xm, sig, jit)
        barrier_sync()
        el_pcie = max_over_ranks(time.perf_counter() - tp0)
        ctx.set_stats(True)
        barrier_sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            ctx.sparse_fit(ks, Xin, Yin, Xm, sig, jit, out=outs)
        barrier_sync()
        el = max_over_ranks(time.perf_counter() - t0)
        st = ctx.stats()
        ctx.set_stats(False)
        outs = None  # (device results freed before the context)
        if ctx is not dctx:
            ctx.close()
        syrk = st.get("other_gemm", {"ms": 0, "launches": 0, "flops": 0})
        # the rank's sigma^-2 Knm^T Knm (+ label row), lower: one split-K launch per streamed row
        # chunk; per launch, the fit's algorithmic flops over its launches and the average device time
        lpf = syrk["launches"] / steps if syrk["launches"] else 0
        t_s = max_over_ranks(syrk["ms"] / syrk["launches"]) if syrk["launches"] else None
        f_syrk = float(len(rows)) * M_ * (M_ + 1) / lpf if lpf else 0.0
        flops = 2.0 * n * M_ * d + n * M_ * (M_ + 1) + 2.0 * M_ ** 3
        c5 = {"workload": "C5: sparse GP fit M=2048 inducing, N=1e6 dense rows, d=64 fp64 GaussianKernel(3,1) "
                          "sigma=0.1 jitter=1e-4 (BASELINE.json configs[4])",
              "metric": "sparse GP fits/sec", "value": steps / el, "unit": "fits/s", "ms_per_step": 1e3 * el / steps,
              "n_gpus": world, "scaling": "strong" if world > 1 else None, "dtype": "f64",
              "note": ("wall time per fit, the rank's rows resident in HBM (device arrays) and the M x M results (Kmm^-1, "
                       "RV, RM) kept there (device destinations); ms_per_step_incl_pcie: rows from and results to "
                       "host memory" if resident else "wall time per fit incl. the upload of the rank's rows (0.5 GB / world)"),
              "inputs_resident": resident,
              "ms_per_step_incl_pcie_upload": 1e3 * el_pcie,
              "fit_tflops_effective": flops / (el / steps) / 1e12,
              "roofline": {"bound": "mfma", "kernel": "syrk_splitk_kernel<double> (sigma^-2 Knm^T Knm, k_syrk.hip)",
                           "achieved": f_syrk / (t_s * 1e-3) / 1e12 if t_s else None, "peak": PEAK_FP64_TFLOPS,
                           "unit": "TFLOP/s", "frac": f_syrk / (t_s * 1e-3) / 1e12 / PEAK_FP64_TFLOPS if t_s else None,
                           "avg_launch_us": 1e3 * t_s if t_s else None, "algorithmic_flops_per_launch": f_syrk,
                           "launches_per_fit": lpf}}
        if world == 1:
            c5["roofline"]["rocprof"] = rocprof_from_profile("c5", ("syrk_splitk_kernel<double>",),
                                                             c5["roofline"]["avg_launch_us"])
        if rank == 0 and world == 1 and args.cpu_n > 0:
            from oracle import oracle as O
            ns = 62500
            O.sparse_fit(ks, Xl[:4096], Yl[:4096], Xm, sig, jit)  # (untimed warm-up)
            t0 = time.perf_counter()
            O.sparse_fit(ks, Xl[:ns], Yl[:ns], Xm, sig, jit)
            dt = time.perf_counter() - t0
            c5["cpu_baseline"] = dict({"value": 1.0 / (dt * n / ns), "unit": "fits/s", "cores": O.num_threads(),
                                       "kind": "port", "extrapolated": True,
                                       "sample": f"1 sparse fit on the first {ns} rows after a warm-up (oracle: Knm build + "
                                                 f"Knm^T Knm + M x M LAPACK inverses) in {dt:.2f} s, scaled LINEARLY in N "
                                                 f"to {n} rows (the M x M part counted 16x: an overestimate of the CPU "
                                                 "rate's cost)"}, **host_info())
        out["C5"] = c5
    except _Skip:
        pass
    except Exception as e:
        out["C5"] = {"error": repr(e)}
    return out


def spawn_ranks(n, argv):
    """`bench.py --gpus N` with no launcher around it (WORLD_SIZE unset): start the N ranks here,
    one child process per GPU, each with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT
    set and the same arguments -- what torch.distributed.run would do -- before this process
    touches the GPU (it never does: no library is loaded here, and nothing is re-executed in
    place).  Rank 0's stdout (the JSON line) is relayed; the other ranks' stdout goes to stderr.
    Returns the exit status: non-zero when any rank fails, when rank 0 printed no JSON line, or
    after GPRX_BENCH_TIMEOUT_S (default 3000 s), the remaining ranks then being killed (their own
    PIDs)."""
    import signal
    import socket
    import subprocess
    import threading
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    lines = []

    def relay(stream):
        for ln in stream:
            sys.stdout.write(ln)
            sys.stdout.flush()
            if ln.startswith("{"):
                lines.append(ln)

    def kill_all(*_):
        for p in procs:
            if p.poll() is None:
                p.kill()

    signal.signal(signal.SIGTERM, lambda *a: (kill_all(), sys.exit(143)))
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GPRX_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno(), text=True))
    th = threading.Thread(target=relay, args=(procs[0].stdout,), daemon=True)
    th.start()
    deadline = time.monotonic() + float(os.environ.get("GPRX_BENCH_TIMEOUT_S", "3000"))
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            log(f"bench.py: rank {bad[0][0]} exited with {bad[0][1]}; stopping the other ranks")
            rc = bad[0][1] if bad[0][1] > 0 else 1
            break
        if all(c == 0 for c in codes):
            break
        if time.monotonic() > deadline:
            log("bench.py: ranks still running at GPRX_BENCH_TIMEOUT_S; stopping them")
            rc = 124
            break
        time.sleep(0.2)
    kill_all()
    for p in procs:
        p.wait()
    th.join(timeout=10)
    if rc == 0 and not lines:
        log("bench.py: rank 0 printed no JSON line")
        rc = 1
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", "--ntrain", dest="n", type=int, default=None,
                    help="training points (--ntrain under torch.distributed.run, whose parser takes --n)")
    ap.add_argument("--d", type=int, default=None)
    ap.add_argument("--predict-q", type=int, default=65536)
    ap.add_argument("--variance-q", type=int, default=None,
                    help="posterior-variance queries (0 = skip; default SURVEY.md 8(d)'s Q = 65536 on one GPU, "
                         "4096 on a sharded fit, whose distributed solve goes chunk by chunk)")
    ap.add_argument("--lml", type=int, default=1, help="also time one log-marginal likelihood + gradient "
                                                        "(BASELINE.json configs[2]); 0 = skip")
    ap.add_argument("--build-iters", type=int, default=3, help="time the covariance build alone (0 = skip)")
    ap.add_argument("--cpu-n", type=int, default=16384, help="N of the CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-lml-ns", default="2048,4096,8192",
                    help="sizes of the CPU LML + gradient baseline, extrapolated cubically to N ('' = skip)")
    ap.add_argument("--cpu-predict-q", type=int, default=4096, help="queries of the CPU predict baseline (0 = skip)")
    ap.add_argument("--mode", choices=["replicas", "dist"], default="dist",
                    help="N>1 headline: one fit whose matrix is sharded over the GPUs (dist, strong "
                         "scaling) or independent fits per GPU (replicas, weak scaling); both are measured")
    ap.add_argument("--configs", type=int, default=1, help="also measure BASELINE configs C2, C4, C5 (0 = skip)")
    ap.add_argument("--dist-lml", type=int, default=0,
                    help="N > 1: also time the LML + gradient on the sharded factor (off by default: not part "
                         "of the headline; rehearsed with two processes on one GPU, DESIGN.md 6)")
    ap.add_argument("--force-dist", action="store_true",
                    help="testing: run the sharded-fit leg (and make it the headline) even at N = 1")
    ap.add_argument("--legs", default="all",
                    help="comma list of the legs to run: " + ",".join(LEGS) + " (profiling passes run one leg per "
                         "process so each rocprof summary holds one configuration: scripts/gpu.sh profile)")
    args = ap.parse_args()
    legs = None if args.legs == "all" else set(args.legs.split(","))
    if legs is not None and not legs <= set(LEGS):
        ap.error(f"unknown legs {sorted(legs - set(LEGS))}")

    def want(leg):
        return legs is None or leg in legs

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # no launcher: start the N ranks ourselves
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    if env_world is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={env_world} from the launcher but --gpus {args.gpus}: they must agree")
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # GPRX_DIST_SHARED_GPU=1: a rehearsal of the N > 1 path on ONE GPU (every rank on device 0,
    # each on its share of the CUs, gloo for the host collectives, the peer context's all-gather
    # for the bootstrap: RCCL refuses two ranks on one device).  Timings are not N-GPU numbers.
    shared = os.environ.get("GPRX_DIST_SHARED_GPU") == "1" and world > 1
    if shared:
        local_rank = 0
    # the library first and no PyTorch at all: the process maps ONE HIP runtime and RCCL,
    # /opt/rocm's (gpr_amd.runtime_info(), reported as "runtime"); the host collectives around
    # the device work (the RCCL unique id, barriers, max over ranks, the peer context's
    # all-gather) are gpr_amd.hostcoll's sockets on the loopback
    import gpr_amd
    from gpr_amd.synth import C3, make_data, make_queries
    gpr_amd.lib()
    if world > 1:
        from gpr_amd.hostcoll import SocketGroup
        dist = SocketGroup.from_env()

    cfg = dict(C3)
    if args.n:
        cfg["n"] = args.n
    if args.d:
        cfg["d"] = args.d
    n, d, m = cfg["n"], cfg["d"], cfg["m"]

    X, Y = make_data(n, d, m)

    def make_model(c):
        mdl = gpr_amd.Model(c, np.float64)
        mdl.set_data(X, Y)
        mdl.set_kernel(cfg["kernel"])
        mdl.set_noise(cfg["sigma"])
        return mdl

    def barrier_sync():
        # (every library call has drained its streams when it returns: the barrier is the
        # host's alone)
        if dist is not None:
            dist.barrier()

    def max_over_ranks(x):
        return x if dist is None else dist.max(x)

    def timed_fits(mdl, c, flags=0):
        """W untimed warmup fits, then exactly K fits between barrier + synchronize; max over ranks."""
        for _ in range(args.warmup):
            mdl.fit(flags)
        c.set_stats(True)
        barrier_sync()
        t0 = time.perf_counter()
        infos = [mdl.fit(flags) for _ in range(args.steps)]
        barrier_sync()
        el = time.perf_counter() - t0
        st = c.stats()
        c.set_stats(False)
        return max_over_ranks(el), infos, st

    # ---- the sharded fit over all ranks (the N > 1 headline) -------------------------------
    dres, dist_error, dctx, transport = None, None, None, None
    if (world > 1 or args.force_dist) and want("c3"):
        try:
            dctx, transport, dist_error = make_dist_context(gpr_amd, dist, rank, world, local_rank, shared)
            dmodel = make_model(dctx)
            el, infos, st = timed_fits(dmodel, dctx, gpr_amd.gprx.FIT_DISTRIBUTED)
            dres = {"elapsed": el, "infos": infos}
            # per-rank evidence for reading a scaling curve: after the timed
            # fits, one more traced fit (untimed) for the measured chain step
            try:
                dres["rank_rec"] = dist_rank_record(dctx, dmodel, transport)
            except Exception as e:
                dres["rank_rec"] = {"rank": rank, "error": repr(e)}
            if args.dist_lml:  # LML + gradient on the sharded factor (row-block partials, one all-reduce)
                dmodel.lml(grad=True, distributed=True)
                barrier_sync()
                tl0 = time.perf_counter()
                dmodel.lml(grad=True, distributed=True)
                dres["lml_ms_wall"] = 1e3 * max_over_ranks(time.perf_counter() - tl0)
            dmodel.close()
        except Exception as e:  # reported; the replicas line stands in
            dist_error = ((dist_error + "; ") if dist_error else "") + repr(e)
            log("distributed fit failed:", dist_error)

    # ---- one independent fit per GPU (the N = 1 headline; the replicas extra for N > 1) -----
    ctx = gpr_amd.Context(local_rank)
    model = make_model(ctx)
    if want("c3"):
        el_r, infos_r, stats = timed_fits(model, ctx)
        replicas = {"value": world * args.steps / el_r, "ms_per_step": 1e3 * el_r / args.steps,
                    "scaling": "weak", "fits_per_step": world}
    else:  # a profiling pass of another leg: one untimed fit for predict / variance
        if want("predict") or want("variance"):
            model.fit()
        el_r, infos_r, stats, replicas = None, [], {}, {"value": None, "ms_per_step": None}

    headline_dist = dres is not None and args.mode == "dist" and (world > 1 or args.force_dist)
    if headline_dist:
        value = args.steps / dres["elapsed"]
        ms_per_step = 1e3 * dres["elapsed"] / args.steps
    else:
        value, ms_per_step = replicas["value"], replicas["ms_per_step"]

    # prediction throughput, query-sharded over the ranks (X and alpha replicated): each rank
    # predicts its contiguous slice of the Q queries; device time of the fused predict
    # kernels, max over ranks
    pred = None
    if args.predict_q > 0 and want("predict"):
        Xq = make_queries(args.predict_q, d)
        lo, hi = gpr_amd.query_shard(args.predict_q, rank, world)
        model.predict(Xq[lo:hi])
        ctx.set_stats(True)
        barrier_sync()
        tq0 = time.perf_counter()
        model.predict(Xq[lo:hi])
        tq = max_over_ranks(time.perf_counter() - tq0)
        ps = ctx.stats().get("predict")
        ctx.set_stats(False)
        pms = max_over_ranks(ps["ms"]) if ps else None
        pred = {"q": args.predict_q, "sharded_over": world,
                "pts_per_s_device": args.predict_q / (pms * 1e-3) if pms else None,
                "pts_per_s_wall_incl_pcie": args.predict_q / tq,
                # F_pred = Q N (2d + 2m) flop
                "roofline": ({"bound": "mfma", "achieved": args.predict_q * n * (2.0 * d + 2.0 * m)
                              / (pms * 1e-3) / 1e12 / world, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                              "frac": args.predict_q * n * (2.0 * d + 2.0 * m) / (pms * 1e-3) / 1e12 / world
                              / PEAK_FP64_TFLOPS} if pms else None)}
        if pms:
            # the same bound for THIS kernel tree: per (query, sample) pair the
            # Gaussian r^2 (d deep) and the periodic statistic (2d deep) on the f64 MFMA units,
            # 2 * 3d flop, plus on the f64 VALU two exps (fexp, 11 ops each) and ~6 ops of leaf
            # scaling, sum and the alpha accumulation; MFMA and f64 VALU do not co-issue
            # (DESIGN.md 4.11), so the two times add.  VALU peak: 78.6 TFLOP/s = 39.3 T FMA/s.
            pairs = float(args.predict_q) * n / world
            t_roof = pairs * 6.0 * d / (PEAK_FP64_TFLOPS * 1e12) + pairs * 28.0 / (PEAK_FP64_TFLOPS / 2 * 1e12)
            pred["roofline_tree"] = {"bound": "mfma+valu (serial)", "t_roof_ms": 1e3 * t_roof,
                                     "t_device_ms": pms, "frac": 1e3 * t_roof / pms,
                                     "mfma_flop_per_pair": 6.0 * d, "valu_ops_per_pair": 28.0}
            # the same tree bound with the f64 VALU at the issue cost the PMC passes measure on
            # this kernel (7.3 cycles per f64 VALU instruction, the spec's rate
            # assumes 4), i.e. at half the spec's FMA rate; the f64 VALU ops per pair after the
            # folded exp: ~25
            t_issue = pairs * 6.0 * d / (PEAK_FP64_TFLOPS * 1e12) + pairs * 25.0 / (PEAK_FP64_TFLOPS / 4 * 1e12)
            pred["roofline_tree_issue"] = {"bound": "mfma + valu at the measured f64 issue cost (serial)",
                                           "t_roof_ms": 1e3 * t_issue, "frac": 1e3 * t_issue / pms,
                                           "valu_ops_per_pair": 25.0, "valu_rate": "half the spec f64 FMA rate"}
            if world == 1:
                pred["rocprof"] = rocprof_from_profile("predict", ("predict_mma_kernel<double, 1, true>",), 1e3 * pms)
                pred["pmc"] = predict_pmc_from_profile()
        if rank == 0 and world == 1 and args.cpu_predict_q > 0:
            try:
                pred["cpu_baseline"] = cpu_predict_baseline(cfg, X, model.alpha(), args.cpu_predict_q)
            except Exception as e:
                log("cpu predict baseline failed:", e)

    # posterior variance (GetCredibleInterval, lib/GaussianProcess.cpp:102-114): k(x,x) - |L^{-1} k_x|^2
    # for Qv queries, query-sharded; the forward solve with Qv right-hand sides on the tile GEMM
    # (Qv N^2 flop) dominates.  Wall time of the call (queries up, variances down: small)
    var = None
    if args.variance_q is None:
        args.variance_q = 65536 if world == 1 else 4096
    if args.variance_q > 0 and want("variance"):
        Xv = make_queries(args.variance_q, d)
        lo, hi = gpr_amd.query_shard(args.variance_q, rank, world)
        model.posterior_cov(Xv[lo:hi], Xv[lo:hi])
        ctx.set_stats(True)
        barrier_sync()
        tv0 = time.perf_counter()
        model.posterior_cov(Xv[lo:hi], Xv[lo:hi])
        tv = max_over_ranks(time.perf_counter() - tv0)
        vs = ctx.stats().get("posterior")
        ctx.set_stats(False)
        # device time of the solve (HIP events around K(x, X), the forward solve and the row
        # dots, on the stream they run on), max over ranks; `ms` is the call's wall time
        vms = max_over_ranks(vs["ms"]) if vs else None
        fl = float(args.variance_q) * n * n
        var = {"q": args.variance_q, "sharded_over": world, "pts_per_s_wall": args.variance_q / tv,
               "ms": 1e3 * tv, "device_ms": vms,
               "pts_per_s_device": (args.variance_q / (vms * 1e-3)) if vms else None,
               "roofline": {"bound": "mfma", "achieved": fl / tv / 1e12 / world,
                            "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                            "frac": fl / tv / 1e12 / world / PEAK_FP64_TFLOPS,
                            "algorithmic_flops": fl, "time": "wall"},
               # the leg's kernels (K(x, X), the recursive forward solve's GEMMs, the row dots) in
               # the committed rocprofv3 summary of this leg
               "rocprof": rocprof_table("variance") if world == 1 else None}

    # log-marginal likelihood + gradient (refit, explicit inverse, fused gradient pass)
    lml = None
    if args.lml and want("lml"):
        model.lml(grad=True)
        ctx.set_stats(True)
        tl0 = time.perf_counter()
        model.lml(grad=True)
        tl = time.perf_counter() - tl0
        ls = ctx.stats()
        ctx.set_stats(False)
        # T_roof = the fit's (B_build + B_solve at HBM rate, n^3/3 at the
        # f64 peak) + potri's 2 n^3 / 3 at the f64 peak + one read of the N(N+1)/2 lower C
        # for the gradient reduction = 56.5 ms; achieved = the LML's algorithmic flops
        # (n^3/3 potrf + n^3/3 trtri + n^3/3 lauum) over the wall time of the call
        t_roof_lml = (fit_roofline_ms(n, d, m) + 1e3 * (2.0 * n ** 3 / 3.0) / (PEAK_FP64_TFLOPS * 1e12)
                      + 1e3 * 8.0 * n * (n + 1) / 2 / (PEAK_HBM_GBS * 1e9))
        lml_flops = float(n) ** 3
        dev_ms = sum(v["ms"] for k, v in ls.items() if k in ("potrf_tiles", "spd_inverse", "other_gemm", "lml_grad", "backsolve"))
        lml = {"ms_wall": 1e3 * tl, "phases_ms": {k: v["ms"] for k, v in ls.items()},
               "device_ms": dev_ms or None,
               "roofline": {"bound": "mfma", "t_roof_ms": t_roof_lml, "t_ms": 1e3 * tl, "time": "wall",
                            "frac": t_roof_lml / (1e3 * tl),
                            "achieved": lml_flops / tl / 1e12, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                            "algorithmic_flops": lml_flops,
                            "note": "factor n^3/3 + triangular inverse n^3/3 (both in one tile launch) + C = U U^T "
                                    "n^3/3, then the gradient pass over the lower C"},
               "rocprof": rocprof_table("lml") if world == 1 else None}
        if lml["rocprof"]:
            # (the committed profile's per-kernel averages summed: one call's device time over
            # the kernels above 1% of the leg)
            lml["roofline"]["rocprof_sum_ms"] = sum(v["avg_us"] for v in lml["rocprof"]["kernels"].values()) / 1e3
        if rank == 0 and world == 1 and args.cpu_lml_ns:
            try:
                lml["cpu_baseline"] = cpu_lml_baseline(cfg, [int(v) for v in args.cpu_lml_ns.split(",")],
                                                       1e3 * tl)
            except Exception as e:
                log("cpu LML baseline failed:", e)

    # the covariance build alone (north_star asks for its HBM GB/s; in the fit it is fused into
    # the factorisation launch as BUILD tasks): the same BUILD tasks with no other task in the
    # ticket list, features resident, device time by HIP events.  Algorithmic bytes per build
    # (SURVEY.md 8(d)): 8 (n d + n (n + 1) / 2) -- X read once, the lower triangle written once.
    build = None
    if args.build_iters > 0 and want("build"):
        try:
            bms = max_over_ranks(ctx.build_time(cfg["kernel"], X, cfg["sigma"], path=0, iters=args.build_iters))
            bbytes = 8.0 * (n * d + n * (n + 1) / 2)
            build = {"ms": bms, "algorithmic_bytes": bbytes, "gbs": bbytes / (bms * 1e-3) / 1e9,
                     "frac_hbm": bbytes / (bms * 1e-3) / 1e9 / PEAK_HBM_GBS,
                     "entries_per_s": n * (n + 1) / 2 / (bms * 1e-3),
                     "kernel": "potrf_tiles_kernel<double, false> with BUILD tasks only (k_ptiles.hip)"}
            # the build is compute-bound for this tree, not HBM-bound: per 128 x 128 lower tile
            # the pair statistics are a 128 x 128 x 3d MFMA product (r^2: d deep, periodic: 2d)
            # and every entry costs two exps (~17 f64 ops each, ocml) plus ~6 ops on the f64
            # VALU, serial with the MFMAs; the stores at HBM rate on top
            ntile = (n // 128) * (n // 128 + 1) / 2
            t_b = (ntile * 2.0 * 128 * 128 * 3 * d / (PEAK_FP64_TFLOPS * 1e12)
                   + ntile * 128 * 128 * 40.0 / (PEAK_FP64_TFLOPS / 2 * 1e12) + bbytes / (PEAK_HBM_GBS * 1e9))
            build["roofline_tree"] = {"bound": "mfma+valu (serial) + hbm stores", "t_roof_ms": 1e3 * t_b,
                                      "frac": 1e3 * t_b / bms}
            if world == 1:
                # the same launch (BUILD tasks only) under rocprof, and its PMC bytes: the twin of
                # `gbs` measured by counters (L2-fabric bytes, FETCH_SIZE x 2 + WRITE_SIZE)
                bk = ("potrf_tiles_kernel<double, false>",)
                build["rocprof"] = rocprof_from_profile("build", bk, 1e3 * bms)
                tr = traffic_from_profile("build", bk)
                build["pmc"] = ({"bytes_per_launch": tr["bytes_per_launch"], "source": tr["source"],
                                 "gbs_pmc": tr["bytes_per_launch"] / (bms * 1e-3) / 1e9} if tr else None)
        except Exception as e:
            log("build timing failed:", e)

    # dominant kernel: the persistent tile-dataflow factorisation, one launch per fit (with
    # the covariance build fused in as BUILD tasks for sum-of-exp-leaf kernel trees).
    # Algorithmic work per launch = n^3/3 (Cholesky) + m n^2 (forward solve of the label
    # rows); the build's work is not counted, so `achieved` understates the launch.  For the
    # sharded fit the launch is each rank's potrf_tiles_kernel<double, true> (device time by
    # HIP events on its stream, max over ranks) and the peak is g GPUs'.
    alg_flops = n ** 3 / 3.0 + m * float(n) ** 2
    if headline_dist:
        avg_ms = max_over_ranks(float(np.mean([i.ms_factor for i in dres["infos"]])))
        infos = dres["infos"]
        kname = "potrf_tiles_kernel<double, true> (one per rank: sharded tile-dataflow build + Cholesky, k_ptiles.hip)"
    else:
        fac = stats.get("potrf_tiles", {"ms": 0, "flops": 0, "launches": 0})
        avg_ms = (fac["ms"] / fac["launches"]) if fac["launches"] else 0.0
        infos = infos_r
        kname = "potrf_tiles_kernel<double> (persistent tile-dataflow covariance build + Cholesky + forward solve, k_ptiles.hip)"
    peak = PEAK_FP64_TFLOPS * (world if headline_dist else 1)
    achieved = (alg_flops / (avg_ms * 1e-3) / 1e12) if avg_ms > 0 else None
    phases = {k: {"ms_per_fit": v["ms"] / args.steps, "launches_per_fit": v["launches"] / args.steps,
                  "tflops": (v["flops"] / (v["ms"] * 1e-3) / 1e12) if v["ms"] and v["flops"] else None,
                  "gbs": (v["bytes"] / (v["ms"] * 1e-3) / 1e9) if v["ms"] and v["bytes"] else None}
              for k, v in stats.items()}
    g_roof = world if headline_dist else 1
    t_roof = fit_roofline_ms(n, d, m, g_roof)
    traffic = traffic_from_profile() if not headline_dist else None
    fit_ms = float(np.median([i.ms_build + i.ms_factor + i.ms_solve for i in infos])) if infos else None

    # every rank's identity and exchange figures (rank 0 prints them): ranks_seen counts the
    # ranks that answered this all-gather, distinct_devices their distinct PCI addresses
    ranks_rec = None
    if world > 1 and dist is not None:
        mine = (dres or {}).get("rank_rec")
        if mine is None:
            try:
                mine = dict(ctx.info())
                mine["note"] = "replicas context (no sharded fit)"
            except Exception as e:
                mine = {"rank": rank, "error": repr(e)}
        ranks_rec = [json.loads(b.decode()) for b in dist.allgather(json.dumps(mine).encode())]
    configs = None
    if args.configs:
        # (the ranks agree whether the sharded fit ran everywhere before the sharded configs use it)
        dist_ok = dres is not None if dist is None else dist.min(1.0 if dres is not None else 0.0) > 0
        configs = run_configs(args, world, rank, local_rank, dctx if dist_ok else None, max_over_ranks,
                              barrier_sync, want)
    if dctx is not None:
        dctx.close()

    if rank == 0:
        cpu = None
        if world == 1 and args.cpu_n > 0 and want("c3"):
            try:
                cpu = cpu_baseline(cfg, args.cpu_n)
            except Exception as e:  # the baseline is reported, never required
                log("cpu baseline failed:", e)
        line = {
            "metric": "GP fits/sec (kernel build + Cholesky + solve), N=16384 d=32 fp64",
            "value": value,
            "unit": "fits/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong" if headline_dist else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SplitMix64 seed 0x47505231, gpr_amd/synth.py)",
            "config": {"workload": "C3: GP fit N=16384 d=32 m=1 Sum(Gaussian(2,0.15)+Periodic(0.1,pi,1)) "
                                   "sigma=1.0 fp64 (BASELINE.json configs[2])",
                       "n": n, "d": d, "m": m, "kernel": cfg["kernel"],
                       "parallelism": (f"sharded: row blocks in cyclic groups over {world} GPUs, tile-dataflow per "
                                       "rank, device-initiated tile pushes over xGMI" if headline_dist
                                       else ("replicas" if world > 1 else "single-gpu"))},
            "roofline": {"bound": "mfma", "kernel": kname,
                         "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                         "frac": achieved / peak if achieved else None,
                         "avg_launch_us": 1e3 * avg_ms if avg_ms else None,
                         "algorithmic_flops_per_launch": alg_flops,
                         # L2-fabric bytes per launch from the committed PMC passes (FETCH_SIZE x 2
                         # for the 16 B/lane operand feed + WRITE_SIZE; MALL hits included, so an
                         # upper bound on HBM bytes), null if none is committed
                         "traffic": (traffic["bytes_per_launch"] if traffic else None),
                         "traffic_kind": "l2_fabric_bytes",
                         "traffic_source": (traffic["source"] if traffic else None),
                         # the same launch in the committed rocprofv3 summary of the C3 leg, and
                         # its matrix-pipe busy fraction from the committed PMC pass
                         "rocprof": (rocprof_from_profile("c3", ("potrf_tiles_kernel<double, false>",),
                                                          1e3 * avg_ms if avg_ms else None)
                                     if not headline_dist else None),
                         "mfma_busy": (mfma_from_profile("c3", ("potrf_tiles_kernel<double, false>",))
                                       if not headline_dist else None)},
            "fit_roofline": {"t_roof_ms": t_roof, "gpus": g_roof, "t_fit_device_ms": fit_ms,
                             "frac": t_roof / fit_ms if fit_ms else None},
            "replicas": replicas if world > 1 else None,
            "dist_error": dist_error,
            "dist_transport": transport,
            # N > 1: how many ranks took part, on how many GPUs, and per rank its device, transport,
            # pushes per fit and the measured diagonal-chain step
            "ranks_seen": (len({r_.get("rank") for r_ in ranks_rec}) if ranks_rec else world),
            "rccl_ranks_seen": (max((r_.get("rccl_count", -1) for r_ in ranks_rec), default=-1) if ranks_rec else None),
            "distinct_devices": (len({r_.get("pci") for r_ in ranks_rec if r_.get("pci")}) if ranks_rec else 1),
            "launcher": ("bench.py spawn" if os.environ.get("GPRX_BENCH_SPAWNED") else
                         ("external (WORLD_SIZE)" if os.environ.get("WORLD_SIZE") else "none (one process)")),
            "ranks": ranks_rec,
            # the HIP runtime, HSA runtime and RCCL this process mapped (one copy each)
            "runtime": gpr_amd.runtime_info(),
            "phases": phases,
            "predict": pred,
            "variance": var,
            "lml_grad": lml,
            "build": build,
            "lml_grad_sharded_ms_wall": (dres or {}).get("lml_ms_wall"),
            "cpu_baseline": cpu,
            "configs": configs,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.close()


if __name__ == "__main__":
    main()
