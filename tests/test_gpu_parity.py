"""GPU parity: libgprx (through the C ABI) against the CPU oracle restatement of the reference.

Tolerances (BASELINE.json north_star): 1e-6 relative (normwise, ||a-b||_inf/||b||_inf) for
fp64 and 1e-3 for fp32 on the fit / predict outputs; entrywise kernel-matrix checks are
tighter since no factorisation is involved.  The reference inverts with LU (dgetrf+dgetri,
include/LAPACKUtils.h:38-56) where libgprx uses Cholesky, so fixtures keep
cond(K + sigma^2 I) well inside 1/tolerance.
"""
import numpy as np
import pytest

from oracle import oracle as O
from tests.helpers import make_data, make_queries, relerr, TOL

pytestmark = pytest.mark.gpu

KERNELS = [
    "GaussianKernel(0.7,1.3,)",
    "PeriodicKernel(0.9,2.5,0.8,)",
    "RationalQuadraticKernel(1.1,0.6,1.5,)",
    "GaussianExpKernel(-0.3,0.1,)",
    "SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))",
    "ProductKernel(GaussianKernel(1.5,1,),PeriodicKernel(1,1.3,0.9,))",
    "SumKernel(GaussianKernel(0.8,1,),WhiteKernel(0.3,))",
    "SumKernel(SumKernel(SumKernel(GaussianKernel(1.2,0.8,),ProductKernel(GaussianKernel(2,0.5,),"
    "PeriodicKernel(0.7,1.7,1.1,))),RationalQuadraticKernel(0.6,0.9,2,)),SumKernel(GaussianKernel(0.4,0.3,),"
    "WhiteKernel(0.05,)))",
]
DTYPES = [np.float64, np.float32]


@pytest.mark.parametrize("ks", KERNELS)
@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("n,d", [(1, 1), (77, 3), (200, 33)])
def test_kernel_matrix(ctx, ks, dtype, n, d):
    X, _ = make_data(n, d, dtype=dtype)
    K = ctx.kernel_matrix(ks, X, dtype)
    R = O.kernel_matrix(ks, X, dtype)
    tol = 1e-12 if dtype == np.float64 else 2e-5
    assert relerr(K, R) <= tol
    assert np.array_equal(K, K.T)


@pytest.mark.parametrize("ks", KERNELS)
def test_deriv_matrix(ctx, ks):
    X, _ = make_data(50, 4)
    D = ctx.deriv_matrix(ks, X)
    R = O.deriv_matrix(ks, X)
    for p in range(R.shape[0]):
        assert relerr(D[p], R[p]) <= 1e-10, p


@pytest.mark.parametrize("ks", KERNELS[:3])
def test_cross_matrix(ctx, ks):
    A, _ = make_data(70, 5)
    B = make_queries(45, 5)
    assert relerr(ctx.cross_matrix(ks, A, B), O.cross_matrix(ks, A, B)) <= 1e-12


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("n", [1, 100, 128, 300, 700])
def test_cholesky(ctx, dtype, n):
    X, _ = make_data(n, 6)
    K = O.kernel_matrix("GaussianKernel(1.1,1,)", X) + 0.1 * np.eye(n)
    L, info = ctx.cholesky(K.astype(dtype))
    assert info == 0
    Lr = np.linalg.cholesky(K)
    assert relerr(L, Lr) <= (1e-10 if dtype == np.float64 else 1e-4)
    assert np.all(np.triu(L, 1) == 0)


def test_cholesky_not_spd(ctx):
    A = np.eye(300)
    A[137, 137] = -1.0
    _, info = ctx.cholesky(A)
    assert info == 138


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("n", [64, 300])
def test_spd_inverse(ctx, dtype, n):
    X, _ = make_data(n, 3)
    K = O.kernel_matrix("GaussianKernel(0.9,1,)", X) + 0.5 * np.eye(n)
    C = ctx.spd_inverse(K.astype(dtype))
    assert relerr(C, np.linalg.inv(K)) <= (1e-10 if dtype == np.float64 else 1e-4)


def _fit(ctx, ks, X, Y, sigma, dtype):
    import gpr_amd
    M = gpr_amd.Model(ctx, dtype)
    M.set_data(X, Y)
    M.set_kernel(ks)
    M.set_noise(sigma)
    info = M.fit()
    return M, info


@pytest.mark.parametrize("ks", KERNELS)
@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("n,d,m", [(200, 2, 1), (517, 8, 3)])
def test_fit_predict(ctx, ks, dtype, n, d, m):
    sigma = 0.5
    X, Y = make_data(n, d, m)
    M, info = _fit(ctx, ks, X.astype(dtype), Y.astype(dtype), sigma, dtype)
    a_ref, C_ref = O.fit(ks, X, Y, sigma, np.float64)
    tol = TOL[np.dtype(dtype)]
    assert relerr(M.alpha(), a_ref) <= tol
    Xq = make_queries(61, d)
    mean, D = M.predict(Xq.astype(dtype), deriv=True)
    mr, Dr = O.predict(ks, X, a_ref, Xq, np.float64, with_deriv=True)
    assert relerr(mean, mr) <= tol
    assert relerr(D, Dr) <= tol
    # logdet against numpy
    K = O.kernel_matrix(ks, X) + sigma * sigma * np.eye(n)
    assert abs(info.logdet - np.linalg.slogdet(K)[1]) <= (1e-8 if dtype == np.float64 else 1e-3) * max(1, abs(info.logdet))


@pytest.mark.parametrize("ks", KERNELS[:5])
def test_posterior_cov_and_core(ctx, ks):
    n, d, sigma = 300, 3, 0.3
    X, Y = make_data(n, d)
    M, _ = _fit(ctx, ks, X, Y, sigma, np.float64)
    _, C_ref = O.fit(ks, X, Y, sigma)
    Xa = make_queries(40, d)
    Xb = Xa[::-1].copy()
    c = M.posterior_cov(Xa, Xb)
    c_ref = O.posterior_cov(ks, X, C_ref, Xa, Xb)
    kab = np.array([O.kernel_eval(ks, a, b, with_grad=False) for a, b in zip(Xa, Xb)])
    # the covariance is a difference of O(1) terms: compare on the scale of k(x,y)
    assert np.max(np.abs(c - c_ref)) <= 1e-6 * max(1.0, np.max(np.abs(kab)))
    C = M.core_matrix()
    assert relerr(C, C_ref) <= 1e-6


@pytest.mark.parametrize("ks", ["SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))",
                                "GaussianKernel(0.7,1.3,)"])
def test_posterior_variance_f32_near_training_points(ctx, ks):
    """fp32 variances k(x,x) - |L^{-1} k_x|^2 at queries within 1e-3 of training samples, where
    the difference cancels hardest (the expanded |u|^2 + |v|^2 - 2 u.v pair statistic
    loses accuracy in fp32, so fp32 models keep the exact-difference build).  Against the oracle's
    fp32 path (K in fp32, inverted in double as include/LAPACKUtils.h:85-97) at the fp32 bar,
    on the scale of k(x,x); pairs (x, y != x) likewise."""
    n, d, sigma = 400, 4, 0.3
    X, Y = make_data(n, d)
    X32, Y32 = X.astype(np.float32), Y.astype(np.float32)
    M, _ = _fit(ctx, ks, X32, Y32, sigma, np.float32)
    _, C_ref = O.fit(ks, X32, Y32, sigma, np.float32)
    rng = np.random.default_rng(7)
    Xa = (X32[rng.choice(n, 64, replace=False)] + 1e-3 * rng.standard_normal((64, d))).astype(np.float32)
    v = M.posterior_cov(Xa, Xa)
    v_ref = O.posterior_cov(ks, X32, C_ref, Xa, Xa, np.float32)
    kaa = max(abs(O.kernel_eval(ks, a, a, with_grad=False)) for a in Xa.astype(np.float64))
    assert np.max(np.abs(v - v_ref)) <= TOL[np.dtype(np.float32)] * max(1.0, kaa)
    Xb = Xa[::-1].copy()
    c = M.posterior_cov(Xa, Xb)
    c_ref = O.posterior_cov(ks, X32, C_ref, Xa, Xb, np.float32)
    assert np.max(np.abs(c - c_ref)) <= TOL[np.dtype(np.float32)] * max(1.0, kaa)
    M.close()


@pytest.mark.parametrize("ks", KERNELS)
def test_lml(ctx, ks):
    n, d, sigma = 150, 2, 0.4
    X, Y = make_data(n, d)
    M, _ = _fit(ctx, ks, X, Y, sigma, np.float64)
    v, g, logdet = M.lml(grad=True)
    vr, gr, det, ldr = O.lml(ks, X, Y, sigma)
    assert abs(v - vr) <= 1e-6 * max(1.0, abs(vr))
    assert abs(logdet - ldr) <= 1e-8 * max(1.0, abs(ldr))
    assert relerr(g, gr) <= 1e-6
    vc, _, _ = M.lml(grad=False, compat=True)
    assert abs(vc - vr) <= 1e-6 * max(1.0, abs(vr))


@pytest.mark.parametrize("ks", ["SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))",
                                "SumKernel(RationalQuadraticKernel(1.1,0.6,1.5,),GaussianExpKernel(-0.3,0.1,))",
                                "PeriodicKernel(0.9,2.5,0.8,)"])
def test_lml_gradient_multi_tile(ctx, ks):
    """The MFMA pair-statistics gradient (k_pairs.hip grad_mma_kernel: r2, S and the
    periodic sum (x-y) sin 2b(x-y) as feature inner products) over many 128 x 128 tiles,
    ragged n, against the oracle's tr((alpha alpha^T - C) dK/dp) (include/Likelihood.h:204-229)."""
    n, d, sigma = 777, 5, 0.7
    X, Y = make_data(n, d)
    M, _ = _fit(ctx, ks, X, Y, sigma, np.float64)
    v, g, _ = M.lml(grad=True)
    vr, gr, _, _ = O.lml(ks, X, Y, sigma)
    assert abs(v - vr) <= 1e-6 * max(1.0, abs(vr))
    assert relerr(g, gr) <= 1e-6


@pytest.mark.parametrize("ks", ["SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))",
                                "GaussianKernel(0.7,1.3,)"])
def test_lml_gradient_f32(ctx, ks):
    """fp32 LML + gradient (the inverse riding along in the fp32 tile factorisation) against
    the oracle in fp32 and fp64, at the fp32 tolerance."""
    n, d, sigma = 600, 4, 0.7
    X, Y = make_data(n, d)
    M, _ = _fit(ctx, ks, X.astype(np.float32), Y.astype(np.float32), sigma, np.float32)
    v, g, _ = M.lml(grad=True)
    vr, gr, _, _ = O.lml(ks, X, Y, sigma)
    assert abs(v - vr) <= 1e-3 * max(1.0, abs(vr))
    assert relerr(g, gr) <= 1e-3


def test_lml_gradient_f32_c3_tree_4096(ctx):
    """The fp32 LML gradient at a C3-shaped size (the C3 tree, d = 32, N = 4096) against the
    oracle's fp32 path (K in float, inverted in double: include/LAPACKUtils.h:85-97) at the
    BASELINE fp32 tolerance.  Measured 5.6e-7 here and 7.4e-6 against the fp64 model at
    N = 16384 (profiles/r03c_lml_f32_error.jsonl)."""
    ks = "SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))"
    n, d, sigma = 4096, 32, 1.0
    X, Y = make_data(n, d)
    X32, Y32 = X.astype(np.float32), Y.astype(np.float32)
    M, _ = _fit(ctx, ks, X32, Y32, sigma, np.float32)
    v, g, _ = M.lml(grad=True)
    vr, gr, _, _ = O.lml(ks, X32, Y32, sigma, np.float32)
    assert abs(v - vr) <= 1e-3 * abs(vr)
    assert relerr(g, gr) <= 1e-3


def test_nonfinite_kernel_matrix(ctx):
    import gpr_amd
    X = np.array([[0.0], [np.inf]])
    with pytest.raises(gpr_amd.GprxError) as e:
        ctx.kernel_matrix("GaussianKernel(1,1,)", X)
    assert "not finite" in str(e.value)


@pytest.mark.parametrize("ks", [KERNELS[0], KERNELS[4]])
def test_set_alpha_restores_predict(ctx, ks):
    """gprx_model_set_alpha (GaussianProcess::Load path, lib/GaussianProcess.cpp:184-268):
    installed regression vectors give bit-identical predictions; the factor-based calls
    need a refit first."""
    import gpr_amd
    from gpr_amd import gprx
    n, d, m, sigma = 260, 3, 2, 0.5
    X, Y = make_data(n, d, m)
    M, _ = _fit(ctx, ks, X, Y, sigma, np.float64)
    Xq = make_queries(33, d)
    mean, D = M.predict(Xq, deriv=True)
    M2 = gprx.Model(ctx, np.float64)
    M2.set_data(X, Y)
    M2.set_kernel(ks)
    M2.set_noise(sigma)
    M2.set_alpha(M.alpha())
    mean2, D2 = M2.predict(Xq, deriv=True)
    assert np.array_equal(mean, mean2) and np.array_equal(D, D2)
    with pytest.raises(gpr_amd.GprxError):
        M2.posterior_cov(Xq, Xq)
    M2.fit()
    assert np.array_equal(M2.alpha(), M.alpha())


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("n", [700, 1536])
def test_distributed_fit_one_rank(dtype, n):
    """The multi-GPU fit (gprx_dist.cpp: row-cyclic sharded storage, per-rank tile launch,
    RCCL transport) on a one-rank RCCL communicator, forced by GPRX_FIT_DISTRIBUTED: same
    alpha / predictions / logdet as the single-GPU path."""
    import gpr_amd
    from gpr_amd import gprx
    ks = KERNELS[4]
    X, Y = make_data(n, 5, 2)
    X, Y = X.astype(dtype), Y.astype(dtype)
    dctx = gpr_amd.Context(0, dist=(0, 1, gpr_amd.unique_id()))
    try:
        Md = gpr_amd.Model(dctx, dtype)
        Md.set_data(X, Y)
        Md.set_kernel(ks)
        Md.set_noise(0.5)
        info_d = Md.fit(gprx.FIT_DISTRIBUTED)
        a_ref, _ = O.fit(ks, X.astype(np.float64), Y.astype(np.float64), 0.5)
        tol = TOL[np.dtype(dtype)]
        assert relerr(Md.alpha(), a_ref) <= tol
        Xq = make_queries(40, 5).astype(dtype)
        mean = Md.predict(Xq)
        assert relerr(mean, O.predict(ks, X.astype(np.float64), a_ref, Xq.astype(np.float64))) <= tol
        K = O.kernel_matrix(ks, X.astype(np.float64)) + 0.25 * np.eye(n)
        assert abs(info_d.logdet - np.linalg.slogdet(K)[1]) <= (1e-8 if dtype == np.float64 else 1e-3) * abs(info_d.logdet)
        Md.close()
    finally:
        dctx.close()


def test_set_data_from_device_memory(ctx):
    """gprx_model_set_data reads host or device memory (include/gprx.h conventions; ADVICE r05:
    it copied with hipMemcpyHostToDevice only): the same data as DeviceArrays of the context gives
    the same fit, bit for bit, as host arrays."""
    import gpr_amd
    ks = "SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))"
    X, Y = make_data(700, 6)
    M_h, _ = _fit(ctx, ks, X, Y, 0.5, np.float64)
    M_d = gpr_amd.Model(ctx, np.float64)
    M_d.set_data(ctx.device_array(X), ctx.device_array(Y))
    M_d.set_kernel(ks)
    M_d.set_noise(0.5)
    M_d.fit()
    assert np.array_equal(M_d.alpha(), M_h.alpha())
    Xq = make_queries(33, 6)
    assert np.array_equal(M_d.predict(Xq), M_h.predict(Xq))
    M_d.close()
    M_h.close()
