"""Tile-engine diagonal 128x128 factor + inverse in isolation (gprx_dev_bench what 11 / 12 / 13:
rank-8 register image / blocked MFMA form / blocked with look-ahead, k_ptiles.hip): us per
factor and phase ticks."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpr_amd  # noqa: E402
from gpr_amd.gprx import lib  # noqa: E402

L = lib()
L.gprx_dev_bench.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64,
                             ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_double)]
ctx = gpr_amd.Context(0)
out = {}
for dt, name in ((1, "f64"), (0, "f32")):
    for what, var in ((11, "rank8"), (12, "blocked"), (13, "lookahead")):
        if dt == 0 and what >= 12:
            continue
        arr = (ctypes.c_double * 10)()
        st = L.gprx_dev_bench(ctx.h, dt, what, 128, 0, 0, 64, ctypes.cast(arr, ctypes.POINTER(ctypes.c_double)))
        if st:
            raise RuntimeError(L.gprx_last_error(ctx.h).decode())
        v = list(arr)
        out[f"{var}_{name}"] = {"us_per_factor": v[0], "us_load": v[1] / 100, "us_ph1": v[2] / 100,
                                "us_ph2": v[3] / 100, "us_ph3": v[4] / 100, "us_total_in_kernel": v[5] / 100}
        if what == 13 and any(v[6:9]):  # GPRX_FACT32_PROF build: fact32 core cycles per factor
            out[f"{var}_{name}"]["fact32_cycles"] = {"pivot": v[6], "panel": v[7], "tail": v[8]}
print(json.dumps(out, indent=1))
