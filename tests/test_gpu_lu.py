"""The LU fallback (k_getrf.hip): a fit whose Cholesky meets a non-positive pivot is redone
with a partial-pivot LU in double -- the reference's default inversion, LAPACK dgetrf_ +
dgetri_ on the matrix cast to double (include/LAPACKUtils.h:38-56, 85-97), reached from
GaussianProcess::InvertKernelMatrix (lib/GaussianProcess.cpp:545-559).

Two kinds of matrices reach it:
* indefinite but well conditioned: RationalQuadraticKernel with a negative alpha (the
  reference validates nothing, include/Kernel.h:799-808) makes K + sigma^2 I indefinite
  (min eigenvalue -0.19, cond 1e4 here).  The LU solution is well defined, so every output
  is compared with the oracle at the BASELINE tolerances;
* numerically singular: sigma = 0 on a dense 1-D grid (tests/GaussianProcessTest.cpp:44 at
  N = 200).  cond(K) ~ 1e20: two LU implementations give different alpha (two LAPACKs
  disagree by 100% here), so the property checked is the one dgetrf_ guarantees, a
  normwise backward error of order eps.
"""
import numpy as np
import pytest

from oracle import oracle as O
from tests.helpers import make_data, make_queries, relerr, TOL

pytestmark = pytest.mark.gpu

INDEF = "RationalQuadraticKernel(1.2,2,-1,)"


def _model(ctx, ks, X, Y, sigma, dtype=np.float64):
    import gpr_amd
    M = gpr_amd.Model(ctx, dtype)
    M.set_data(X, Y)
    M.set_kernel(ks)
    M.set_noise(sigma)
    return M


@pytest.mark.parametrize("n,d,m", [(700, 3, 2), (1500, 3, 1), (260, 3, 1)])
def test_lu_fallback_indefinite_f64(ctx, n, d, m):
    sigma = 0.3
    X, Y = make_data(n, d, m)
    K = O.kernel_matrix(INDEF, X) + sigma * sigma * np.eye(n)
    assert np.linalg.eigvalsh(K)[0] < 0  # indefinite: the Cholesky must fail
    M = _model(ctx, INDEF, X, Y, sigma)
    info = M.fit()
    assert info.method == 1 and info.info > 0
    a_ref, C_ref = O.fit(INDEF, X, Y, sigma)
    assert relerr(M.alpha(), a_ref) <= 1e-6
    Xq = make_queries(64, d)
    mean, D = M.predict(Xq, deriv=True)
    mr, Dr = O.predict(INDEF, X, a_ref, Xq, with_deriv=True)
    assert relerr(mean, mr) <= 1e-6 and relerr(D, Dr) <= 1e-6
    sign, ld = np.linalg.slogdet(K)
    assert abs(info.logdet - ld) <= 1e-9 * max(1.0, abs(ld))
    cov = M.posterior_cov(Xq, Xq[::-1].copy())
    cov_ref = O.posterior_cov(INDEF, X, C_ref, Xq, Xq[::-1].copy())
    assert np.max(np.abs(cov - cov_ref)) <= 1e-6 * max(1.0, np.max(np.abs(cov_ref)))
    assert relerr(M.core_matrix(), C_ref) <= 1e-6
    M.close()


def test_lu_fallback_lml(ctx):
    n, d, sigma = 700, 3, 0.3
    X, Y = make_data(n, d, 1)
    M = _model(ctx, INDEF, X, Y, sigma)
    v, g, logdet = M.lml(grad=True)
    vr, gr, det, ldr = O.lml(INDEF, X, Y, sigma)
    assert abs(logdet - ldr) <= 1e-9 * max(1.0, abs(ldr))
    assert abs(v - vr) <= 1e-6 * max(1.0, abs(vr))  # det < 0 or > 0: the reference's clamp included
    assert relerr(g, gr) <= 1e-6
    vc, _, _ = M.lml(grad=False, compat=True)
    assert abs(vc - vr) <= 1e-6 * max(1.0, abs(vr))
    M.close()


def test_lu_fallback_f32(ctx):
    """fp32 GP: K evaluated in float, factored in double (lu_invert<float>, :85-97)."""
    n, d, sigma = 700, 3, 0.3
    X, Y = make_data(n, d, 1)
    X32, Y32 = X.astype(np.float32), Y.astype(np.float32)
    M = _model(ctx, INDEF, X32, Y32, sigma, np.float32)
    info = M.fit()
    assert info.method == 1
    a_ref, _ = O.fit(INDEF, X32, Y32, sigma, np.float32)
    assert relerr(M.alpha(), a_ref) <= 1e-3
    Xq = make_queries(40, d).astype(np.float32)
    assert relerr(M.predict(Xq), O.predict(INDEF, X32, a_ref, Xq, np.float32)) <= 1e-3
    M.close()


def test_no_lu_fallback_flag(ctx):
    import gpr_amd
    from gpr_amd import gprx
    X, Y = make_data(300, 3, 1)
    M = _model(ctx, INDEF, X, Y, 0.3)
    with pytest.raises(gpr_amd.GprxError) as e:
        M.fit(gprx.FIT_NO_LU_FALLBACK)
    assert e.value.status == 2  # NOT_SPD
    M.close()


def test_lu_after_cholesky_model_switches_back(ctx):
    """A model refitted with a positive definite kernel goes back to the Cholesky factor."""
    X, Y = make_data(400, 3, 1)
    M = _model(ctx, INDEF, X, Y, 0.3)
    assert M.fit().method == 1
    M.set_kernel("GaussianKernel(0.7,1.3,)")
    info = M.fit()
    assert info.method == 0
    a_ref, C_ref = O.fit("GaussianKernel(0.7,1.3,)", X, Y, 0.3)
    assert relerr(M.alpha(), a_ref) <= 1e-6
    Xq = make_queries(20, 3)
    cov = M.posterior_cov(Xq, Xq)
    assert np.max(np.abs(cov - O.posterior_cov("GaussianKernel(0.7,1.3,)", X, C_ref, Xq, Xq))) <= 1e-6
    M.close()


@pytest.mark.parametrize("N", [50, 200])
def test_lu_fallback_singular_sigma0(ctx, N):
    """tests/GaussianProcessTest.cpp:35-76 at N = 50 and 200 (sigma = 0, Gaussian(2.889)):
    the Cholesky of the numerically singular K fails and the LU solves it with a normwise
    backward error of order eps, as dgetrf_ + dgetrs_ guarantee (scipy's LU reaches 1e-17
    here; the reference's own route, the explicit dgetri_ inverse times Y, only 1e-11)."""
    ks = "GaussianKernel(2.889,1,)"
    x = np.array([[i * 2 * np.pi / N] for i in range(N)])
    y = np.sin(x)
    M = _model(ctx, ks, x, y, 0.0)
    info = M.fit()
    assert info.method == 1
    a = M.alpha()
    K = O.kernel_matrix(ks, x)
    berr = np.max(np.abs(K @ a - y)) / (np.max(np.abs(K).sum(1)) * np.max(np.abs(a)))
    assert berr <= 1e-15, berr
    M.close()


def test_exactly_singular_raises(ctx):
    """A zero kernel (RationalQuadraticKernel with scale 0, no validation in the reference)
    and sigma = 0: K = 0, the LU's first pivot is exactly zero."""
    import gpr_amd
    X, Y = make_data(150, 2, 1)
    M = _model(ctx, "RationalQuadraticKernel(0,1,1,)", X, Y, 0.0)
    with pytest.raises(gpr_amd.GprxError) as e:
        M.fit()
    assert e.value.status == 3  # SINGULAR
    M.close()


def test_svd_inversion_methods(ctx):
    """JacobiSVD / BDCSVD (lib/GaussianProcess.cpp:564-592) form core = V S^{-1} U^T, the exact
    inverse of a nonsingular K; GPRX_FIT_FORCE_LU produces that matrix through the LU in double.
    Restated with numpy's SVD (LAPACK gesdd) on an ill-conditioned K."""
    from gpr_amd import gprx
    n, d, sigma = 400, 2, 1e-3
    ks = "GaussianKernel(0.9,1.0,)"
    X, Y = make_data(n, d, 1)
    K = O.kernel_matrix(ks, X) + sigma * sigma * np.eye(n)
    U, S, Vt = np.linalg.svd(K)
    core = Vt.T @ np.diag(1.0 / S) @ U.T
    a_svd = core @ Y
    M = _model(ctx, ks, X, Y, sigma)
    info = M.fit(gprx.FIT_FORCE_LU)
    assert info.method == 1
    cond = S[0] / S[-1]
    tol = max(1e-9, 50 * cond * np.finfo(np.float64).eps)
    assert relerr(M.alpha(), a_svd) <= tol
    Xq = make_queries(30, d)
    assert relerr(M.predict(Xq), O.cross_matrix(ks, Xq, X) @ a_svd) <= tol
    v, g, ld = M.lml(grad=True, force_lu=True)
    assert abs(ld - np.linalg.slogdet(K)[1]) <= 1e-8 * abs(ld)
    M.close()
