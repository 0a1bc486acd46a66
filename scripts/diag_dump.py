import sys, os, numpy as np
sys.path.insert(0, os.getcwd())
import gpr_amd
from tests.test_gpu_diag import _factor, _sparse_normal_block
ctx = gpr_amd.Context(0)
A = _sparse_normal_block()
out = {"A": A}
for v in (0, 1, 2):
    L, Li, info = _factor(ctx, v, A)
    out[f"L{v}"] = L; out[f"Li{v}"] = Li; out[f"info{v}"] = info
np.savez("gpurun_out/diag_dump.npz", **out)
print("ok")
