"""A/B of the tile factorisation's memory feed: device time of one potrf_tiles launch (N = 16384,
f64, gprx_dev_bench what 9) as shipped, and with GPRX_PT_VARIANT=64 (every update streams the
same L2-resident operand tiles: wrong numbers, same task graph, same MFMA work).  The difference
bounds what any cut of the update operands' L2-miss traffic can buy.  Run once per variant:
    GPRX_PT_VARIANT=64 python scripts/traffic_ab.py
"""
import ctypes, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpr_amd
from gpr_amd.gprx import lib

L = lib()
L.gprx_dev_bench.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64,
                             ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_double)]
ctx = gpr_amd.Context(0)
n = int(os.environ.get("AB_N", "16384"))
iters = int(os.environ.get("AB_ITERS", "5"))
ms = ctypes.c_double()
st = L.gprx_dev_bench(ctx.h, 1, 9, n, 0, 0, iters, ctypes.byref(ms))
# variant 64 makes the matrix indefinite: a NOT_SPD status is expected and harmless for timing
print(json.dumps({"n": n, "variant": int(os.environ.get("GPRX_PT_VARIANT", "0")), "status": st,
                  "ms": ms.value, "tflops": n ** 3 / 3 / ms.value / 1e9}), flush=True)
