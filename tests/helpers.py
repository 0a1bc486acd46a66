"""Shared test helpers: deterministic inputs (gpr_amd/synth.py) and the parity metric."""
import numpy as np

from gpr_amd.synth import SEED, splitmix64, uniform, make_data, make_queries  # noqa: F401


def relerr(a, b, tiny=1e-300):
    """Normwise relative error ||a-b||_inf / max(||b||_inf, tiny)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), tiny))


TOL = {np.dtype(np.float64): 1e-6, np.dtype(np.float32): 1e-3}
