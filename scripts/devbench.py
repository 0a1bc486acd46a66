"""Isolated kernel timings through gprx_dev_bench (include/gprx_dev.h)."""
import ctypes, sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpr_amd
from gpr_amd.gprx import lib

L = lib()
L.gprx_dev_bench.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64,
                             ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_double)]
ctx = gpr_amd.Context(0)


def run(dt, what, M, N=0, K=0, iters=10):
    ms = ctypes.c_double()
    st = L.gprx_dev_bench(ctx.h, dt, what, M, N, K, iters, ctypes.byref(ms))
    if st:
        raise RuntimeError(L.gprx_last_error(ctx.h).decode())
    return ms.value


cases = sys.argv[1] if len(sys.argv) > 1 else "all"
res = {}
F64, F32 = 1, 0
if cases in ("all", "diag"):
    for dt in (F64, F32):
        ms = run(dt, 0, 128, iters=50)
        res[f"diag128_{'f64' if dt else 'f32'}_us"] = ms * 1e3

if cases in ("all", "diag", "diagprof"):
    for dt in (F64, F32):
        arr = (ctypes.c_double * 5)()
        st = L.gprx_dev_bench(ctx.h, dt, 6, 128, 0, 0, 20, ctypes.cast(arr, ctypes.POINTER(ctypes.c_double)))
        if st:
            raise RuntimeError(L.gprx_last_error(ctx.h).decode())
        res[f"diagprof_{'f64' if dt else 'f32'}_ticks"] = dict(zip(["load", "solve", "update", "store", "total"], list(arr)))

if cases in ("all", "gemm"):
    for (M, N, K, low) in [(16384, 16384, 256, 1), (16384, 16384, 512, 1), (8192, 8192, 256, 1), (16384, 128, 128, 0),
                           (16384, 256, 256, 0), (8192, 8192, 1024, 0), (4096, 4096, 4096, 0)]:
        ms = run(F64, 2 if low else 1, M, N, K, iters=5)
        fl = 2.0 * K * ((N * (N + 1) / 2 + (M - N) * N) if low else M * N)
        res[f"gemm_f64_{M}x{N}x{K}{'_low' if low else ''}"] = {"ms": ms, "tflops": fl / ms / 1e9}
    for (M, N, K, low) in [(16384, 16384, 256, 1), (8192, 8192, 1024, 0)]:
        ms = run(F32, 2 if low else 1, M, N, K, iters=5)
        fl = 2.0 * K * ((N * (N + 1) / 2 + (M - N) * N) if low else M * N)
        res[f"gemm_f32_{M}x{N}x{K}{'_low' if low else ''}"] = {"ms": ms, "tflops": fl / ms / 1e9}
if cases in ("all", "graph"):
    for n in (4096, 16384):
        res[f"potrf_graph_f64_{n}_ms"] = run(F64, 7, n, iters=3)
    res["backsolve_graph_f64_16384_ms"] = run(F64, 8, 16384, iters=5)

if cases in ("all", "potrf"):
    for n in (4096, 16384):
        for what, name in ((3, "single"), (4, "lookahead")):
            ms = run(F64, what, n, iters=2)
            res[f"potrf_f64_{n}_{name}"] = {"ms": ms, "tflops": n ** 3 / 3 / ms / 1e9}
    ms = run(F64, 5, 16384, iters=3)
    res["backsolve_f64_16384_ms"] = ms
print(json.dumps(res, indent=1))
