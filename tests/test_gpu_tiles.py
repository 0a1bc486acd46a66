"""GPU tests of the tile-dataflow factorisation (k_ptiles.hip) and the flag-chained back
substitution (k_bsolve.hip) at sizes where the schedule uses W-deep update chunks, several
panels and the label row block -- the production path of GaussianProcess::Initialize
(lib/GaussianProcess.cpp:118-130) at BASELINE.json scale.

Oracle: numpy Cholesky for the factor, the CPU restatement (oracle/, LU inverse in fp64 as
the reference's lapack::lu_invert) for alpha, and -- at the full C3 size, where the oracle's
O(N^3) LU would take minutes -- the size-independent residual property
||(K + s^2 I) alpha - Y||_inf / ||Y||_inf with K rebuilt by the (separately parity-tested)
kernel-matrix path.
"""
import numpy as np
import pytest

import gpr_amd
from oracle import oracle as O
from tests.helpers import make_data, make_queries, relerr, TOL

pytestmark = pytest.mark.gpu


def _spd(n, seed, dtype=np.float64):
    rng = np.random.default_rng(seed)
    B = rng.standard_normal((n, n))
    return (B @ B.T / n + np.eye(n)).astype(dtype)


@pytest.mark.parametrize("n", [1029, 2048, 3000])
def test_tile_cholesky_f64(ctx, n):
    A = _spd(n, n)
    L, info = ctx.cholesky(A.copy())
    assert info == 0
    assert relerr(L, np.linalg.cholesky(A)) <= 1e-12
    assert np.all(np.triu(L, 1) == 0)


@pytest.mark.parametrize("n", [1100, 2304])
def test_tile_cholesky_f32(ctx, n):
    A = _spd(n, n + 1)
    L, info = ctx.cholesky(A.astype(np.float32))
    assert info == 0
    assert relerr(L, np.linalg.cholesky(A)) <= 1e-4


@pytest.mark.parametrize("bad", [0, 700, 1999, 2047])
def test_tile_cholesky_not_spd_terminates(ctx, bad):
    """A non-SPD pivot anywhere (first block, mid-panel, last block) must report the first
    failing column and still drain the device scheduler (no hang, no timeout code)."""
    A = np.eye(2048)
    A[bad, bad] = -1.0
    _, info = ctx.cholesky(A)
    assert info == bad + 1


def test_tile_cholesky_nan_terminates(ctx):
    A = _spd(1536, 3)
    A[900, 900] = np.nan
    _, info = ctx.cholesky(A)
    assert info > 0  # NaN pivot is "not > 0": reported, and the launch completes


@pytest.mark.parametrize("ks", ["GaussianKernel(0.7,1.3,)",
                                "SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))"])
@pytest.mark.parametrize("n,d,m", [(2100, 6, 1), (1500, 4, 3)])
def test_tile_fit_predict(ctx, ks, n, d, m):
    sigma = 0.5
    X, Y = make_data(n, d, m)
    M = gpr_amd.Model(ctx, np.float64)
    M.set_data(X, Y)
    M.set_kernel(ks)
    M.set_noise(sigma)
    info = M.fit()
    a_ref, _ = O.fit(ks, X, Y, sigma, np.float64)
    assert relerr(M.alpha(), a_ref) <= TOL[np.dtype(np.float64)]
    Xq = make_queries(97, d)
    assert relerr(M.predict(Xq), O.predict(ks, X, a_ref, Xq, np.float64)) <= TOL[np.dtype(np.float64)]
    K = O.kernel_matrix(ks, X) + sigma * sigma * np.eye(n)
    assert abs(info.logdet - np.linalg.slogdet(K)[1]) <= 1e-8 * max(1.0, abs(info.logdet))
    M.close()


MEAN_KERNELS = ["GaussianKernel(0.7,1.3,)", "PeriodicKernel(0.9,2.5,0.8,)", "RationalQuadraticKernel(1.1,0.6,1.5,)",
                "GaussianExpKernel(-0.3,0.1,)",
                "SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))",
                "ProductKernel(GaussianKernel(1.5,1,),PeriodicKernel(1,1.3,0.9,))",
                "SumKernel(GaussianKernel(0.8,1,),WhiteKernel(0.3,))"]


@pytest.mark.parametrize("ks", MEAN_KERNELS)
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("n,d,q", [(300, 3, 1), (777, 33, 300)])
def test_mean_predict_and_build_paths(ctx, ks, dtype, n, d, q):
    """Mean-only prediction and the covariance build take the MFMA pair-statistics kernels
    (k_pairs.hip) for White-free trees, the direct kernels otherwise; both against the oracle."""
    sigma = 0.5
    X, Y = make_data(n, d, 1)
    M = gpr_amd.Model(ctx, dtype)
    M.set_data(X.astype(dtype), Y.astype(dtype))
    M.set_kernel(ks)
    M.set_noise(sigma)
    M.fit()
    a_ref, _ = O.fit(ks, X, Y, sigma, np.float64)
    tol = TOL[np.dtype(dtype)]
    assert relerr(M.alpha(), a_ref) <= tol
    Xq = make_queries(q, d)
    assert relerr(M.predict(Xq.astype(dtype)), O.predict(ks, X, a_ref, Xq, np.float64)) <= tol
    M.close()


def test_c3_full_size_residual(ctx):
    """BASELINE.json configs[2] at full size (N = 16384, d = 32, Sum(Gaussian + Periodic),
    sigma = 1): the fit's alpha solves (K + s^2 I) alpha = Y to near machine precision."""
    from gpr_amd.synth import C3
    n, d, ks, sigma = C3["n"], C3["d"], C3["kernel"], C3["sigma"]
    X, Y = make_data(n, d, 1)
    M = gpr_amd.Model(ctx, np.float64)
    M.set_data(X, Y)
    M.set_kernel(ks)
    M.set_noise(sigma)
    info = M.fit()
    alpha = M.alpha()
    K = ctx.kernel_matrix(ks, X)
    K[np.diag_indices(n)] += sigma * sigma
    r = K @ alpha - Y
    assert np.max(np.abs(r)) / np.max(np.abs(Y)) <= 1e-10
    # the Jensen bound of SURVEY.md §8(d) keeps the log-determinant finite and positive
    assert 0.0 < info.logdet <= n * (0.15 ** 2 + 0.1 ** 2) + n * np.log(1.0 + 1e-12) + 1.0
    M.close()


@pytest.mark.parametrize("ks", ["SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))",
                                "GaussianExpKernel(-0.3,0.1,)", "RationalQuadraticKernel(1.1,0.6,1.5,)"])
def test_predict_at_training_points(ctx, ks):
    """Queries ON training points (and offset copies of them): the MFMA predict's pair
    statistics r2 = |x~|^2 + |y~|^2 - 2 x~.y~ and S round to tiny negatives there and are
    used unclamped (k_pairs.h pair_stats_nc); the predictions must still match the oracle's
    direct differences (lib/GaussianProcess.cpp:54-61)."""
    sigma = 0.7
    n, d = 640, 9
    X, Y = make_data(n, d, 1)
    M = gpr_amd.Model(ctx, np.float64)
    M.set_data(X, Y)
    M.set_kernel(ks)
    M.set_noise(sigma)
    M.fit()
    a_ref, _ = O.fit(ks, X, Y, sigma, np.float64)
    Xq = np.concatenate([X[::3], X[:50] + 1e-9])
    p = M.predict(Xq)
    assert np.all(np.isfinite(p))
    assert relerr(p, O.predict(ks, X, a_ref, Xq, np.float64)) <= 1e-6
    M.close()


_TALL_CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import gpr_amd
from gpr_amd.synth import make_data, make_queries
ctx = gpr_amd.Context(0)
X, Y = make_data(8192, 8)
M = gpr_amd.Model(ctx, np.float64)
M.set_data(X, Y)
M.set_kernel("GaussianKernel(1.3,1,)")
M.set_noise(0.5)
M.fit()
np.save(sys.argv[2], M.posterior_cov(make_queries(4096, 8), make_queries(4096, 8)))
"""


def test_posterior_tall_gemms_match_128_tiles(tmp_path):
    """The posterior variance's bulk GEMMs on the 256 x 128 tile (k_syrk.hip gemm_tall_kernel,
    its refill DMAs spread behind the MFMAs for f64) against the 128 x 128 tile
    (GPRX_GEMM_TALL=0) at a size that routes to them (Q = 4096, N = 8192): the same sums in the
    same k order, so the variances agree to the last bit."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = []
    for tag, env in (("on", {}), ("off", {"GPRX_GEMM_TALL": "0"})):
        f = tmp_path / f"v_{tag}.npy"
        r = subprocess.run([sys.executable, "-c", _TALL_CHILD, root, str(f)], env=dict(os.environ, **env),
                           capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(np.load(f))
    assert np.array_equal(outs[0], outs[1])


@pytest.mark.gpu
def test_posterior_repeatable_in_place_solves():
    """The row solves' diagonal-block products run in place (k_predict.hip trsm_rows: R_k =
    R_k Linv_k^T); launch_gemm_nt keeps them on whole-row tiles (k_potrf.hip), since with 64 x 64
    tiles the workgroup of columns 64..127 could read columns its neighbour had already
    overwritten -- an intermittent error in a 64-query block (seen once in ~150 processes at
    N = 8192, Q = 4096).  Repeated variances of one fit agree to the last bit."""
    from gpr_amd.synth import make_data, make_queries
    ctx = gpr_amd.Context(0)
    X, Y = make_data(8192, 8)
    M = gpr_amd.Model(ctx, np.float64)
    M.set_data(X, Y)
    M.set_kernel("GaussianKernel(1.3,1,)")
    M.set_noise(0.5)
    M.fit()
    Q = make_queries(4096, 8)
    v0 = M.posterior_cov(Q, Q)
    for _ in range(6):
        assert np.array_equal(M.posterior_cov(Q, Q), v0)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [np.float64, np.float32])
def test_paths_repeatable(dt):
    """Every multi-workgroup path gives the same bits when repeated on the same model: the
    fused fit (paired updates, balanced TRSM tiles), the LML + gradient (identity rows paired,
    C = U U^T, the gradient pass), the mean and the variance.  Guards the class of the in-place
    race above: a cross-workgroup read-after-write shows up as a call that differs."""
    from gpr_amd.synth import make_data, make_queries
    ctx = gpr_amd.Context(0)
    X, Y = make_data(6144, 8)
    M = gpr_amd.Model(ctx, dt)
    M.set_data(X, Y)
    M.set_kernel("SumKernel(GaussianKernel(1.3,1,),PeriodicKernel(0.7,1.1,2.0,))"
                 if dt == np.float64 else "GaussianKernel(1.3,1,)")
    M.set_noise(0.5)
    Q = make_queries(2048, 8)
    outs = []
    for _ in range(3):
        M.fit()
        v, g, ld = M.lml(grad=True)
        outs.append((M.alpha().copy(), np.asarray(M.predict(Q)).copy(), np.asarray(M.posterior_cov(Q, Q)).copy(),
                     np.float64(v), np.asarray(g).copy(), np.float64(ld)))
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert np.array_equal(a, b)


@pytest.mark.gpu
def test_lml_gradient_fallback_repeatable():
    """The gradient pass for trees the MFMA statistics do not carry (a product of leaves:
    k_lml.hip lml_grad_kernel) sums per-workgroup slots in a fixed order instead of atomics:
    repeated LML + gradient calls give the same bits."""
    from gpr_amd.synth import make_data
    ctx = gpr_amd.Context(0)
    X, Y = make_data(2048, 4)
    M = gpr_amd.Model(ctx, np.float64)
    M.set_data(X, Y)
    M.set_kernel("ProductKernel(GaussianKernel(1.5,1,),PeriodicKernel(1,1.3,0.9,))")
    M.set_noise(0.5)
    M.fit()
    v0, g0, l0 = M.lml(grad=True)
    for _ in range(4):
        v, g, ld = M.lml(grad=True)
        assert v == v0 and ld == l0 and np.array_equal(np.asarray(g), np.asarray(g0))
