"""The PRODUCTION covariance build, entrywise against the oracle.

The default fit never materialises K by itself: for sum-of-exp-leaf trees (Gaussian,
GaussianExp, Periodic -- C3's class) the tiles are built by the BUILD tasks inside the
persistent tile factorisation (k_ptiles.hip), for the other trees without a White leaf by
kbuild_mma_kernel (k_pairs.hip), both from per-sample features whose inner products give
r2 = |x~|^2 + |y~|^2 - 2 x~.y~ and the periodic statistic.  gprx_dev_build_matrix runs
exactly those device paths alone (path 0: the BUILD tasks with no other task in the ticket
list; path 1: kbuild_mma_kernel) and returns the tile lower triangle, so the values the
factorisation starts from are compared entry by entry with the reference's pair loop
(lib/GaussianProcess.cpp:384-402 + noise :375-381, restated in oracle/).  Offset and
wide-range inputs exercise the cancellation in the r2 expansion; non-finite inputs must be
rejected as the reference rejects them (:399-401).
"""
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.helpers import make_data, make_queries, relerr

pytestmark = pytest.mark.gpu

FUSED = [  # sum-of-exp-leaf trees: path 0 (and 1)
    "GaussianKernel(0.7,1.3,)",
    "PeriodicKernel(0.9,2.5,0.8,)",
    "GaussianExpKernel(-0.3,0.1,)",
    "SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))",
]
UNFUSED = [  # MFMA build as its own kernel: path 1 only
    "RationalQuadraticKernel(1.1,0.6,1.5,)",
    "ProductKernel(GaussianKernel(1.5,1,),PeriodicKernel(1,1.3,0.9,))",
    "SumKernel(RationalQuadraticKernel(1,0.3,1,),GaussianKernel(1.2,0.8,))",
]


def _inputs(kind, n, d):
    X, _ = make_data(n, d)
    if kind == "unit":
        return X
    if kind == "offset":  # far from the origin: the expansion is centred on sample 0
        return X + 1e3
    if kind == "wide":  # wide range: |x~|^2 ~ 2500 d
        return X * 50.0
    if kind == "mixed":  # per-dimension scales over 4 decades
        return X * np.logspace(-2, 2, d)[None, :]
    raise ValueError(kind)


def _ref(ks, X, sigma, dtype=np.float64):
    return O.kernel_matrix(ks, X, dtype) + dtype(sigma) * dtype(sigma) * np.eye(X.shape[0], dtype=dtype)


@pytest.mark.parametrize("kind", ["unit", "offset", "wide", "mixed"])
@pytest.mark.parametrize("ks", FUSED)
@pytest.mark.parametrize("path", [0, 1])
def test_build_fused_trees(ctx, ks, kind, path):
    n, d, sigma = 300, 7, 0.3
    X = _inputs(kind, n, d)
    K = ctx.build_matrix(ks, X, sigma, path)
    assert relerr(K, _ref(ks, X, sigma)) <= 1e-12
    assert np.array_equal(np.diag(K), np.diag(_ref(ks, X, sigma)))  # r2 = S = 0 exactly on the diagonal


@pytest.mark.parametrize("kind", ["unit", "offset", "wide"])
@pytest.mark.parametrize("ks", UNFUSED)
def test_build_unfused_trees(ctx, ks, kind):
    n, d, sigma = 260, 5, 0.4
    X = _inputs(kind, n, d)
    assert relerr(ctx.build_matrix(ks, X, sigma, 1), _ref(ks, X, sigma)) <= 1e-12
    with pytest.raises(Exception):  # the fused path does not carry these trees
        ctx.build_matrix(ks, X, sigma, 0)


@pytest.mark.parametrize("n,d", [(1, 1), (129, 33), (1000, 32)])
def test_build_c3_shapes(ctx, n, d):
    ks = FUSED[3]
    X, _ = make_data(n, d)
    assert relerr(ctx.build_matrix(ks, X, 1.0, 0), _ref(ks, X, 1.0)) <= 1e-12


@pytest.mark.parametrize("path", [0, 1])
def test_build_time_hook(ctx, path):
    """gprx_dev_build_time (bench.py's build GB/s) runs the same launches and reports time."""
    X, _ = make_data(1000, 32)
    ms = ctx.build_time(FUSED[3], X, 1.0, path, iters=2)
    assert 0.0 < ms < 1e3


def test_build_breathing_raw_scale(ctx):
    """The reference's own 1-D breathing signal (tests/data/breathing1D.mat) at its raw
    amplitude, as sample coordinates: time-delay embedding x_i = (s_i, s_{i+1}, s_{i+2})."""
    from tests.golden.make_golden import read_matrixio
    s = read_matrixio(os.path.join(os.path.dirname(__file__), "golden", "breathing1D.mat"))[0]
    X = np.stack([s[:600], s[1:601], s[2:602]], axis=1)
    for ks in (FUSED[0], FUSED[3]):
        assert relerr(ctx.build_matrix(ks, X, 0.1, 0), _ref(ks, X, 0.1)) <= 1e-12


def test_build_f32(ctx):
    X, _ = make_data(400, 9)
    X = X.astype(np.float32)
    for ks in FUSED:
        K = ctx.build_matrix(ks, X, 0.5, 0, np.float32)
        assert relerr(K, _ref(ks, X, 0.5, np.float32)) <= 2e-5


@pytest.mark.parametrize("bad", [np.nan, np.inf, -np.inf])
@pytest.mark.parametrize("ks", [FUSED[0], FUSED[3], UNFUSED[0]])
@pytest.mark.parametrize("row", [0, 77, 199])
def test_fit_rejects_nonfinite_inputs(ctx, ks, bad, row):
    """A NaN/Inf sample makes the reference's K non-finite and Initialize throw
    (lib/GaussianProcess.cpp:399-401); the feature-based build must not clamp it away."""
    import gpr_amd
    X, Y = make_data(200, 4)
    X[row, 2] = bad
    M = gpr_amd.Model(ctx, np.float64)
    M.set_data(X, Y)
    M.set_kernel(ks)
    M.set_noise(0.5)
    with pytest.raises(gpr_amd.GprxError) as e:
        M.fit()
    assert "not finite" in str(e.value)
    with pytest.raises(gpr_amd.GprxError):
        ctx.build_matrix(ks, X, 0.5, 1)


def test_predict_nonfinite_query_propagates(ctx):
    """Predict does not validate its input in the reference: a NaN query gives a NaN mean
    (Kx(NaN) = NaN), it must not come back as a finite value."""
    import gpr_amd
    ks = FUSED[3]
    X, Y = make_data(300, 4)
    M = gpr_amd.Model(ctx, np.float64)
    M.set_data(X, Y)
    M.set_kernel(ks)
    M.set_noise(0.5)
    M.fit()
    Xq = make_queries(10, 4)
    Xq[3, 1] = np.nan
    mean = M.predict(Xq)
    assert np.isnan(mean[3, 0])
    assert np.all(np.isfinite(np.delete(mean, 3, axis=0)))


def test_sparse_rejects_nonfinite_inputs(ctx):
    X, Y = make_data(500, 3)
    X[10, 0] = np.nan
    with pytest.raises(Exception) as e:
        ctx.sparse_fit("GaussianKernel(1,1,)", X, Y, X[::10].copy() + 0.01, 0.1, 1e-4)
    assert "not finite" in str(e.value)


def test_fexp_accuracy(ctx):
    """The epilogues' table-driven f64 exp (gprx_internal.h fexp) against numpy's exp: <= 2 ulp
    over the arguments the kernels produce (c r2, c S <= 0, down to the underflow), 0 below
    -745.5, NaN kept."""
    import ctypes
    from gpr_amd.gprx import lib
    L = lib()
    L.gprx_dev_fexp.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    rng = np.random.default_rng(7)
    x = np.concatenate([-np.abs(rng.standard_normal(200000)) * 3, -rng.random(200000) * 745.0,
                        rng.random(20000) * 20, np.linspace(-708.5, -700, 5000), [0.0, -0.0, -1e-300, -746.0, np.nan]])
    y = np.empty_like(x)
    assert L.gprx_dev_fexp(ctx.h, x.ctypes.data, x.size, y.ctypes.data) == 0
    ref = np.exp(x)
    fin = np.isfinite(x) & (x > -708)  # normal results: error in ulps of the reference
    ulp = np.abs(y[fin] - ref[fin]) / np.spacing(ref[fin])
    assert ulp.max() <= 2.0, ulp.max()
    sub = np.isfinite(x) & (x <= -708) & (x >= -745.0)  # subnormal range: absolute error
    assert np.max(np.abs(y[sub] - ref[sub])) <= 4 * np.spacing(0.0)
    assert y[-2] == 0.0 and np.isnan(y[-1])
