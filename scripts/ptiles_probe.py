"""GPU probe of the tile-dataflow potrf: correctness vs numpy and timing vs the stream path."""
import ctypes, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import gpr_amd
from gpr_amd.gprx import lib

L = lib()
L.gprx_dev_bench.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64,
                             ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_double)]
ctx = gpr_amd.Context(0)
res = {}
rng = np.random.default_rng(1)
for n in [int(x) for x in os.environ.get("PT_NS", "128,256,640,1024,2048").split(",")]:
    B = rng.standard_normal((n, n))
    A = B @ B.T / n + np.eye(n)
    Lr = np.linalg.cholesky(A)
    Lg = ctx.cholesky(A.copy())[0]
    Lg = np.tril(Lg)
    err = np.max(np.abs(Lg - Lr)) / np.max(np.abs(Lr))
    res[f"chol_{n}_relerr"] = float(err)
    print(n, err, flush=True)


def run(what, M, iters=3):
    ms = ctypes.c_double()
    st = L.gprx_dev_bench(ctx.h, 1, what, M, 0, 0, iters, ctypes.byref(ms))
    if st:
        raise RuntimeError(L.gprx_last_error(ctx.h).decode())
    return ms.value


for n in [int(x) for x in os.environ.get("PT_TN", "4096,16384").split(",")]:
    for what, name in ((9, "tiles"), (4, "streams")):
        ms = run(what, n)
        res[f"potrf_{n}_{name}"] = {"ms": ms, "tflops": n ** 3 / 3 / ms / 1e9}
        print(n, name, ms, flush=True)
print(json.dumps(res, indent=1))
