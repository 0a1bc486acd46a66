"""Kernels with no device form (the reference's virtual Kernel<T>::operator(), include/
Kernel.h:52-59): the caller evaluates K, the query kernel vectors and the derivative
matrices; libgprx factors, solves and reduces on the GPU (gprx_model_set_kernel_matrix,
gprx_model_predict_kx, gprx_model_posterior_cov_kx, gprx_model_lml_dk; k_hostk.hip).
Checked against numpy solves of the same matrices (a Matern-3/2 kernel, which has no device
form), and against the device kernel for a host-evaluated Gaussian."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.helpers import make_data, make_queries, relerr

pytestmark = pytest.mark.gpu


class Matern32:
    """k = s^2 (1 + sqrt(3) r / l) exp(-sqrt(3) r / l); parameters (l, s)."""

    def __init__(self, l, s):
        self.l, self.s = l, s

    def _r(self, A, B):
        return np.sqrt(np.maximum(np.sum((A[:, None, :] - B[None, :, :]) ** 2, axis=-1), 0.0))

    def __call__(self, A, B):
        a = np.sqrt(3.0) * self._r(A, B) / self.l
        return self.s ** 2 * (1 + a) * np.exp(-a)

    def gradient(self, A, B):
        a = np.sqrt(3.0) * self._r(A, B) / self.l
        e = np.exp(-a)
        dl = self.s ** 2 * a * a * e / self.l  # d/dl of s^2 (1 + a) e^{-a}, a = sqrt3 r / l
        ds = 2 * self.s * (1 + a) * e
        return np.stack([dl, ds])


class HostGauss:
    def __init__(self, sig, sc):
        self.sig, self.sc = sig, sc

    def __call__(self, A, B):
        r2 = np.sum((A[:, None, :] - B[None, :, :]) ** 2, axis=-1)
        return self.sc ** 2 * np.exp(-0.5 * r2 / self.sig ** 2)

    def gradient(self, A, B):
        r2 = np.sum((A[:, None, :] - B[None, :, :]) ** 2, axis=-1)
        e = np.exp(-0.5 * r2 / self.sig ** 2)
        return np.stack([self.sc ** 2 * r2 / self.sig ** 3 * e, 2 * self.sc * e])


def _model(ctx, k, X, Y, sigma, dtype=np.float64):
    import gpr_amd
    M = gpr_amd.Model(ctx, dtype)
    M.set_data(X, Y)
    M.set_kernel(k)
    M.set_noise(sigma)
    M.fit()
    return M


def test_matern_host_kernel_vs_numpy():
    import gpr_amd
    n, d, m, sigma = 300, 3, 2, 0.3
    X, Y = make_data(n, d, m)
    k = Matern32(0.6, 1.2)
    ctx = gpr_amd.Context(0)
    try:
        M = _model(ctx, k, X, Y, sigma)
        Kn = k(X, X) + sigma ** 2 * np.eye(n)
        aref = np.linalg.solve(Kn, Y)
        assert relerr(M.alpha(), aref) <= 1e-10
        Xq = make_queries(40, d)
        mean, D = M.predict(Xq, deriv=True)
        Kx = k(Xq, X)
        assert relerr(mean, Kx @ aref) <= 1e-10
        Dref = np.stack([-(Xq[i][None, :] - X).T @ (Kx[i][:, None] * aref) for i in range(40)])
        assert relerr(D, Dref) <= 1e-10
        Xb = make_queries(40, d)[::-1].copy()
        cov = M.posterior_cov(Xq, Xb)
        Ka, Kb = k(Xq, X), k(Xb, X)
        cref = np.array([k(Xq[i:i + 1], Xb[i:i + 1])[0, 0] for i in range(40)]) - np.sum(
            Ka * np.linalg.solve(Kn, Kb.T).T, axis=1)
        assert np.max(np.abs(cov - cref)) <= 1e-9
        M.close()
        # LML value + gradient (m = 1)
        M1 = _model(ctx, k, X, Y[:, :1], sigma)
        v, g, ld = M1.lml(grad=True)
        g2 = M1.lml(grad=True)[1]  # fixed-order sums (k_hostk.hip dk_grad_sum_kernel): the same bits
        assert np.array_equal(np.asarray(g), np.asarray(g2))
        a1 = np.linalg.solve(Kn, Y[:, 0])
        ldref = np.linalg.slogdet(Kn)[1]
        vref = -0.5 * Y[:, 0] @ a1 - 0.5 * ldref - n / 2 * np.log(2 * np.pi)
        C = np.linalg.inv(Kn)
        gref = np.array([0.5 * np.sum((np.outer(a1, a1) - C) * Dp) for Dp in k.gradient(X, X)])
        assert abs(ld - ldref) <= 1e-9 * abs(ldref)
        assert abs(v - vref) <= 1e-9 * abs(vref)
        assert relerr(g, gref) <= 1e-8
        M1.close()
    finally:
        ctx.close()


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_host_gaussian_matches_device_gaussian(dtype):
    import gpr_amd
    n, d, sigma = 500, 4, 0.4
    X, Y = make_data(n, d, 1)
    X, Y = X.astype(dtype), Y.astype(dtype)
    ctx = gpr_amd.Context(0)
    try:
        Mh = _model(ctx, HostGauss(0.8, 1.1), X, Y, sigma, dtype)
        Md = _model(ctx, "GaussianKernel(0.8,1.1,)", X, Y, sigma, dtype)
        tol = 1e-10 if dtype == np.float64 else 2e-3
        assert relerr(Mh.alpha(), Md.alpha()) <= tol
        Xq = make_queries(30, d).astype(dtype)
        assert relerr(Mh.predict(Xq), Md.predict(Xq)) <= tol
        if dtype == np.float64:
            vh, gh, _ = Mh.lml(grad=True)
            vd, gd, _ = Md.lml(grad=True)
            assert abs(vh - vd) <= 1e-8 * abs(vd)
            assert relerr(gh, gd) <= 1e-7
        Mh.close()
        Md.close()
    finally:
        ctx.close()


def test_host_kernel_lu_fallback():
    """A caller-evaluated indefinite K takes the LU fallback like a device kernel."""
    import gpr_amd
    n, d = 260, 3
    X, Y = make_data(n, d, 1)
    ks = "RationalQuadraticKernel(1.2,2,-1,)"  # indefinite (tests/test_gpu_lu.py)
    Kf = O.kernel_matrix(ks, X)
    assert np.linalg.eigvalsh(Kf + 0.09 * np.eye(n))[0] < 0
    ctx = gpr_amd.Context(0)
    try:
        M = gpr_amd.Model(ctx, np.float64)
        M.set_data(X, Y)
        M.set_kernel(lambda A, B: O.cross_matrix(ks, A, B) if A is not B else Kf)
        M.set_noise(0.3)
        info = M.fit()
        assert info.method == 1
        aref = np.linalg.solve(Kf + 0.09 * np.eye(n), Y)
        assert relerr(M.alpha(), aref) <= 1e-8
        Xq = make_queries(20, d)
        Kq = O.cross_matrix(ks, Xq, X)
        assert relerr(M.predict(Xq), Kq @ aref) <= 1e-8
        cov = M.posterior_cov(Xq, Xq)
        kk = np.array([O.cross_matrix(ks, Xq[i:i + 1], Xq[i:i + 1])[0, 0] for i in range(20)])
        cref = kk - np.sum(Kq * np.linalg.solve(Kf + 0.09 * np.eye(n), Kq.T).T, axis=1)
        assert np.max(np.abs(cov - cref)) <= 1e-7 * max(1.0, np.max(np.abs(cref)))
        M.close()
    finally:
        ctx.close()
