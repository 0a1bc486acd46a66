"""One dev-bench case: python devbench_one.py <what> <M> [N K iters dtype(1=f64)]."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpr_amd
from gpr_amd.gprx import lib
L = lib()
L.gprx_dev_bench.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64,
                             ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_double)]
a = [int(x) for x in sys.argv[1:]] + [0] * 6
what, M, N, K, iters, dt = a[0], a[1], a[2], a[3], a[4] or 2, (a[5] if len(sys.argv) > 6 else 1)
ctx = gpr_amd.Context(0)
ms = ctypes.c_double()
st = L.gprx_dev_bench(ctx.h, dt, what, M, N, K, iters, ctypes.byref(ms))
print("status", st, "ms", ms.value, flush=True)
