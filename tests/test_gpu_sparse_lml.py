"""Sparse GP log-marginal likelihood on the GPU (gprx_sparse_lml) vs the oracle's literal
restatement of SparseGaussianLogLikelihood::GetValueAndParameterDerivatives
(include/SparseLikelihood.h:231-344: N x N C_inv by EfficientInversion, the A_p stack, the
long-double EfficientDeterminant with its clamps).  The device evaluates the same quantities
in O(N M^2) (Woodbury; gprx_api.cpp sparse_lml_impl).  Sparse-path parity is unpinned by the
reference's own tests (tests/SparseInferenceTest.cpp:486-489 are disabled): the oracle is the
checker, cross-checked against numpy in tests/test_oracle_numpy.py.

Tolerances: value and gradient normwise relative error <= 1e-6 (fp64), 1e-3 (fp32); the
oracle's literal N x N form is itself only accurate to cond(C) * eps, so the inputs keep
cond(K + jitter I) moderate (jitter 1e-3)."""
import numpy as np
import pytest

import gpr_amd
from oracle import oracle as O
from tests.helpers import make_data, relerr, TOL

pytestmark = pytest.mark.gpu

CASES = [
    # (kernel, dtype, jitter, sigma): the MFMA gradient path (sums of Gaussian / GaussianExp /
    # RQ / one Periodic) and the VALU path (products, White)
    ("GaussianKernel(0.7,1.3,)", np.float64, 1e-3, 0.3),
    ("SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))", np.float64, 1e-3, 0.5),
    ("RationalQuadraticKernel(1.1,0.6,1.5,)", np.float64, 1e-3, 0.4),
    ("GaussianExpKernel(-0.3,0.2,)", np.float64, 1e-3, 0.4),
    ("ProductKernel(GaussianKernel(0.9,1.1,),RationalQuadraticKernel(1,0.8,2,))", np.float64, 1e-3, 0.4),
    ("SumKernel(GaussianKernel(0.8,1,),WhiteKernel(0.3,))", np.float64, 1e-3, 0.4),
    ("GaussianKernel(0.7,1.3,)", np.float32, 0.5, 2.0),
]


def _inputs(n, d, M, dtype):
    X, Y = make_data(n, d, 1)
    Xm = X[:: n // M][:M].copy()
    return X.astype(dtype), Y[:, 0].astype(dtype), Xm.astype(dtype)


def _tol_value(v_ref, dtype):
    return TOL[np.dtype(dtype)] * max(1.0, abs(v_ref))


@pytest.mark.parametrize("ks,dtype,jitter,sigma", CASES)
@pytest.mark.parametrize("chunk", [None, 128])
def test_sparse_lml_vs_oracle(ctx, monkeypatch, ks, dtype, jitter, sigma, chunk):
    if chunk:
        monkeypatch.setenv("GPRX_SPARSE_CHUNK", str(chunk))
    n, d, M = 600, 3, 40
    X, y, Xm = _inputs(n, d, M, dtype)
    v, g, ld = ctx.sparse_lml(ks, X, y, Xm, sigma, jitter, dtype)
    vr, gr, det_r, ld_r = O.sparse_lml(ks, X, y, Xm, sigma, jitter, dtype)
    tol = TOL[np.dtype(dtype)]
    assert abs(v - vr) <= _tol_value(vr, dtype), (v, vr)
    assert abs(ld - ld_r) <= tol * max(1.0, abs(ld_r)), (ld, ld_r)
    assert g.shape == gr.shape
    assert relerr(g, gr) <= tol, (g, gr)
    # compat mode reproduces the reference's long-double determinant product; inside its
    # range it agrees with the exact value
    vc, gc, _ = ctx.sparse_lml(ks, X, y, Xm, sigma, jitter, dtype, compat=True)
    assert abs(vc - vr) <= _tol_value(vr, dtype)
    # (the VALU path for products / White sums its tiles with atomics: last-bit differences)
    assert relerr(gc, g) <= 1e-12


def test_sparse_lml_value_only_and_repeat(ctx):
    """operator() (include/SparseLikelihood.h:148-216) is the value alone; repeated calls give
    bit-identical results (fixed summation orders)."""
    ks = "SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))"
    X, y, Xm = _inputs(900, 5, 60, np.float64)
    v0, g0, _ = ctx.sparse_lml(ks, X, y, Xm, 0.5, 1e-3)
    v1, g1, _ = ctx.sparse_lml(ks, X, y, Xm, 0.5, 1e-3)
    v2, g2, _ = ctx.sparse_lml(ks, X, y, Xm, 0.5, 1e-3, grad=False)
    assert v0 == v1 == v2 and g2 is None
    assert np.array_equal(g0, g1)


def test_sparse_lml_compat_clamp(ctx):
    """At N = 20000, sigma = 0.1 the reference's product det(Kmm^-1) sigma^{2N} det(B) underflows
    long double (log10 ~ -40000): cp is clamped to -log(LDBL_MIN)/2 (:305-314); the exact mode
    keeps the true log-determinant."""
    ks = "GaussianKernel(0.7,1.3,)"
    X, y, Xm = _inputs(20000, 3, 64, np.float64)
    v, _, ld = ctx.sparse_lml(ks, X, y, Xm, 0.1, 1e-3, grad=False)
    vc, _, ldc = ctx.sparse_lml(ks, X, y, Xm, 0.1, 1e-3, grad=False, compat=True)
    assert ld == ldc and ld < np.log(np.finfo(np.longdouble).tiny)
    ldbl_min_log = np.log(np.finfo(np.longdouble).tiny)
    # exact: df - ld/2 - ct; compat: df + (-0.5 log(LDBL_MIN)) - ct
    assert abs((vc - v) - (-0.5 * ldbl_min_log + 0.5 * ld)) <= 1e-8 * abs(vc)


def test_sparse_lml_gradient_fd_large(ctx):
    """Beyond the oracle's reach (N = 50000, M = 512, d = 16, several row chunks): the gradient
    against Richardson-extrapolated central differences of the device value."""
    n, d, M = 50000, 16, 512
    X, y, Xm = _inputs(n, d, M, np.float64)
    # cond(Kmm + jitter I) ~ 6e3: the value's rounding stays far below the difference quotient's
    # resolution (at jitter 1e-4, length scale 1.7 cond ~ 3e5 and a float64 numpy evaluation of the
    # same formulas differs from its own differences by 2e-6)
    sig, sc, sigma, jitter = 1.0, 0.9, 0.3, 1e-3

    def val(sg, s):
        return ctx.sparse_lml(f"GaussianKernel({sg!r},{s!r},)", X, y, Xm, sigma, jitter, grad=False)[0]

    _, g, _ = ctx.sparse_lml(f"GaussianKernel({sig!r},{sc!r},)", X, y, Xm, sigma, jitter)

    def cd(f, x, h):
        return (f(x + h) - f(x - h)) / (2 * h)

    for k, (f, x) in enumerate([(lambda t: val(t, sc), sig), (lambda t: val(sig, t), sc)]):
        h = 1e-2 * x
        fd = (4 * cd(f, x, h / 2) - cd(f, x, h)) / 3
        assert abs(g[k] - fd) <= 1e-6 * max(1.0, abs(fd)), (k, g[k], fd)


def test_sparse_lml_errors(ctx):
    X, y, Xm = _inputs(300, 3, 20, np.float64)
    with pytest.raises(gpr_amd.GprxError, match="no inducing samples"):
        ctx.sparse_lml("GaussianKernel(1,1,)", X, y, Xm[:0], 0.3, 1e-3)
    Xb = X.copy()
    Xb[17, 1] = np.nan
    with pytest.raises(gpr_amd.GprxError, match="not finite"):
        ctx.sparse_lml("GaussianKernel(1,1,)", Xb, y, Xm, 0.3, 1e-3)
    with pytest.raises(gpr_amd.GprxError, match="sigma must be positive"):
        ctx.sparse_lml("GaussianKernel(1,1,)", X, y, Xm, 0.0, 1e-3)
