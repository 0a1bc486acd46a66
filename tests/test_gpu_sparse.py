"""Sparse GP (subset of regressors) on the GPU vs the oracle restatement of
SparseGaussianProcess::PreComputeRegression (include/SparseGaussianProcess.h:274-313).

The device computes RV = S^{-1} sigma^-2 Knm^T Y and RM = S^{-1} from one Cholesky of
S = Kmm + jitter I + sigma^-2 Knm^T Knm (the reference's Kinv (sigma^-2 K Sigma Knm^T Y) and
Kinv (K Sigma K) Kinv are algebraically these), streaming Knm in
row chunks.  The oracle's sparse path is pinned by the reference's own sparse checks,
tests/SparseInferenceTest.cpp Test1-3 (disabled in its main, :486-489, restated as KATs in
tests/test_oracle_kats.py); the device runs the same configurations below
(test_sparse_reference_*).  Inducing points are rows i*(N/M) of X."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.helpers import make_data, make_queries, relerr, TOL

pytestmark = pytest.mark.gpu

CASES = [
    ("GaussianKernel(0.7,1.3,)", np.float64, 1e-4, 0.3),
    ("SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))", np.float64, 1e-4, 0.5),
    ("RationalQuadraticKernel(1.1,0.6,1.5,)", np.float64, 1e-3, 0.3),
    # fp32: the reference itself is only meaningful when cond(S) * eps32 is small (at jitter
    # 0.1, sigma 0.5 the oracle's own fp32 result is 11% off its fp64 one); cond(S) = 2.7e3 here
    ("GaussianKernel(0.7,1.3,)", np.float32, 0.5, 5.0),
]


def _inputs(n, d, M, m, dtype):
    X, Y = make_data(n, d, m)
    Xm = X[:: n // M][:M].copy()
    return X.astype(dtype), Y.astype(dtype), Xm.astype(dtype)


@pytest.mark.parametrize("ks,dtype,jitter,sigma", CASES)
@pytest.mark.parametrize("chunk", [None, 64])
def test_sparse_fit(ctx, monkeypatch, ks, dtype, jitter, sigma, chunk):
    if chunk:
        monkeypatch.setenv("GPRX_SPARSE_CHUNK", str(chunk))
    n, d, M, m = 700, 3, 40, 2
    X, Y, Xm = _inputs(n, d, M, m, dtype)
    Kinv, RV, RM = ctx.sparse_fit(ks, X, Y, Xm, sigma, jitter, dtype)
    Ki_r, RV_r, RM_r = O.sparse_fit(ks, X, Y, Xm, sigma, jitter, dtype)
    tol = TOL[np.dtype(dtype)]  # BASELINE.json's bar: 1e-6 fp64, 1e-3 fp32
    assert relerr(Kinv, Ki_r) <= tol
    assert relerr(RV, RV_r) <= tol
    assert relerr(RM, RM_r) <= tol


def test_sparse_predict_through_dense_model(ctx):
    """SparseGaussianProcess::Predict (:86-92) = Kx^T RV over the inducing points: served by a
    resident model holding the inducing points and RV (gprx_model_set_alpha)."""
    import gpr_amd
    ks = "GaussianKernel(0.7,1.3,)"
    X, Y, Xm = _inputs(1000, 4, 50, 1, np.float64)
    _, RV, _ = ctx.sparse_fit(ks, X, Y, Xm, 0.3, 1e-4)
    Mdl = gpr_amd.Model(ctx, np.float64)
    Mdl.set_data(Xm, np.zeros((Xm.shape[0], 1)))
    Mdl.set_kernel(ks)
    Mdl.set_noise(0.0)
    Mdl.set_alpha(RV)
    Xq = make_queries(77, 4)
    mean = Mdl.predict(Xq)
    _, RV_r, _ = O.sparse_fit(ks, X, Y, Xm, 0.3, 1e-4)
    ref = O.predict(ks, Xm, RV_r, Xq)
    assert relerr(mean, ref) <= 1e-6


def test_sparse_bad_sigma(ctx):
    import gpr_amd
    X, Y, Xm = _inputs(100, 2, 10, 1, np.float64)
    with pytest.raises(gpr_amd.GprxError) as e:
        ctx.sparse_fit("GaussianKernel(1,1,)", X, Y, Xm, 0.0, 1e-4)
    assert "sigma must be positive" in str(e.value)


@pytest.mark.parametrize("ks", ["GaussianKernel(0.7,1.3,)",
                                "SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))"])
def test_sparse_fit_multi_tile(ctx, monkeypatch, ks):
    """Several 128-tiles of inducing points (M = 300: diagonal, off-diagonal and partial
    tiles), several streamed chunks with split-K partials (P > 1) and a ragged last chunk.
    Same tolerance as test_sparse_fit: the oracle follows the reference's Kinv-based formulas,
    the device one Cholesky of S (algebraically equal)."""
    monkeypatch.setenv("GPRX_SPARSE_CHUNK", "2048")
    n, d, M, m = 5000, 8, 300, 1
    X, Y, Xm = _inputs(n, d, M, m, np.float64)
    Kinv, RV, RM = ctx.sparse_fit(ks, X, Y, Xm, 0.3, 1e-3, np.float64)
    Ki_r, RV_r, RM_r = O.sparse_fit(ks, X, Y, Xm, 0.3, 1e-3, np.float64)
    tol = TOL[np.dtype(np.float64)] * 10
    assert relerr(Kinv, Ki_r) <= tol
    assert relerr(RV, RV_r) <= tol
    assert relerr(RM, RM_r) <= tol
    assert np.array_equal(Kinv, Kinv.T) and np.array_equal(RM, RM.T)


@pytest.mark.parametrize("ks", [CASES[0][0], CASES[1][0]])
def test_sparse_operator_on_device(ctx, ks):
    """SparseGaussianProcess::operator()(x,y) = k(x,y) - Kx^T Kinv Ky + Kx^T RM Ky
    (include/SparseGaussianProcess.h:94-106) from the resident W = Kinv - RM
    (gprx_model_set_sparse_cov), batched over q pairs, vs the oracle's matrices in numpy."""
    import gpr_amd
    n, d, M, m = 900, 3, 60, 1
    X, Y, Xm = _inputs(n, d, M, m, np.float64)
    Kinv, RV, RM = ctx.sparse_fit(ks, X, Y, Xm, 0.3, 1e-4)
    Ki_r, RV_r, RM_r = O.sparse_fit(ks, X, Y, Xm, 0.3, 1e-4)
    S = gpr_amd.Model(ctx, np.float64)
    S.set_data(Xm, Y[:: n // M][:M])
    S.set_kernel(ks)
    S.set_alpha(RV)
    S.set_sparse_cov(Kinv - RM)
    Xa, Xb = make_queries(150, d), make_queries(150, d)[::-1].copy()
    cov = S.posterior_cov(Xa, Xb)
    Ka, Kb = O.cross_matrix(ks, Xa, Xm), O.cross_matrix(ks, Xb, Xm)
    kab = np.array([O.cross_matrix(ks, Xa[i:i + 1], Xb[i:i + 1])[0, 0] for i in range(150)])
    ref = kab - np.sum(Ka * ((Ki_r - RM_r) @ Kb.T).T, axis=1)
    assert np.max(np.abs(cov - ref)) <= 1e-8 * max(1.0, np.max(np.abs(ref)))
    S.close()


def test_sparse_fit_rccl_one_rank():
    """gprx_sparse_fit on an RCCL context: the dense rows are the rank's shard and the partial
    normal equations [Kmn; Y^T][Kmn; Y^T]^T are summed by ncclAllReduce (SURVEY.md 8(e)
    "Sparse fit"); on one rank the result equals the local fit."""
    import gpr_amd
    ks = CASES[0][0]
    n, d, M, m = 800, 3, 48, 1
    X, Y, Xm = _inputs(n, d, M, m, np.float64)
    lctx = gpr_amd.Context(0)
    dctx = gpr_amd.Context(0, dist=(0, 1, gpr_amd.unique_id()))
    try:
        Kl, RVl, RMl = lctx.sparse_fit(ks, X, Y, Xm, 0.3, 1e-4)
        Kd, RVd, RMd = dctx.sparse_fit(ks, X, Y, Xm, 0.3, 1e-4)
        assert relerr(RVd, RVl) <= 1e-12 and relerr(RMd, RMl) <= 1e-12 and relerr(Kd, Kl) <= 1e-12
    finally:
        dctx.close()
        lctx.close()


def test_sparse_lml_rccl_one_rank():
    """gprx_sparse_lml on an RCCL context (rows sharded; normal equations, data terms and the
    N x M gradient partials all-reduced): on one rank it equals the local call."""
    import gpr_amd
    ks = CASES[1][0]
    n, d, M, m = 800, 3, 48, 1
    X, Y, Xm = _inputs(n, d, M, m, np.float64)
    lctx = gpr_amd.Context(0)
    dctx = gpr_amd.Context(0, dist=(0, 1, gpr_amd.unique_id()))
    try:
        vl, gl, ldl = lctx.sparse_lml(ks, X, Y, Xm, 0.5, 1e-3)
        vd, gd, ldd = dctx.sparse_lml(ks, X, Y, Xm, 0.5, 1e-3)
        assert vd == vl and ldd == ldl and np.array_equal(gd, gl)
    finally:
        dctx.close()
        lctx.close()


def test_sparse_fit_device_array_inputs(ctx):
    """X and Y already in HBM (the library's own device buffers, gprx_device_alloc): read without a
    PCIe copy (unified addressing picks the copy's direction), the same bits as from host arrays;
    the buffers round-trip, a reshaped view shares its base's memory, m = 1 labels as a vector."""
    ks = "GaussianKernel(0.7,1.3,)"
    X, Y, Xm = _inputs(3000, 4, 64, 1, np.float64)
    host = ctx.sparse_fit(ks, X, Y, Xm, 0.3, 1e-4)
    Xd, Yd = ctx.device_array(X), ctx.device_array(Y)
    assert np.array_equal(Xd.numpy(), X) and Xd.shape == X.shape
    dev = ctx.sparse_fit(ks, Xd, Yd, Xm, 0.3, 1e-4)
    for a, b in zip(host, dev):
        assert np.array_equal(a, b)
    Yv = ctx.device_array(np.ascontiguousarray(Y[:, 0]))  # (n,) -> reshaped to (n, 1) inside
    dev1 = ctx.sparse_fit(ks, Xd, Yv, Xm, 0.3, 1e-4)
    for a, b in zip(host, dev1):
        assert np.array_equal(a, b)
    assert Yv.reshape(-1, 1).data_ptr() == Yv.data_ptr()
    with pytest.raises(TypeError):
        ctx.sparse_fit(ks, Xd, ctx.device_array(Y.astype(np.float32)), Xm, 0.3, 1e-4)
    # results kept in HBM (DeviceArray destinations: no PCIe copy), the same bits; repeated calls
    # reuse the context's sparse state (and a different shape in between re-sizes it)
    import gpr_amd
    outs = tuple(gpr_amd.DeviceArray.empty(ctx, shp) for shp in ((64, 64), (64, 1), (64, 64)))
    X2, Y2, Xm2 = _inputs(1500, 4, 200, 1, np.float64)
    fctx = gpr_amd.Context(0)  # (a fresh context: the reference bits for the other shape)
    try:
        fresh = fctx.sparse_fit(ks, X2, Y2, Xm2, 0.3, 1e-2)
    finally:
        fctx.close()
    for _ in range(2):
        ctx.sparse_fit(ks, Xd, Yd, Xm, 0.3, 1e-4, out=outs)
        for a, b in zip(host, outs):
            assert np.array_equal(a, b.numpy())
        other = ctx.sparse_fit(ks, X2, Y2, Xm2, 0.3, 1e-2)
        for a, b in zip(fresh, other):
            assert np.array_equal(a, b)
    with pytest.raises(ValueError):
        ctx.sparse_fit(ks, Xd, Yd, Xm, 0.3, 1e-4, out=(outs[1], outs[1], outs[2]))


def test_sparse_fit_device_resident_inputs(ctx):
    """X and Y already in HBM (a torch CUDA tensor's memory): the library reads them without a
    PCIe copy (unified addressing picks the copy's direction) and returns the same bits as from
    host arrays.  (Skipped in a process where this library initialised the device first: the
    PyTorch wheel's bundled HIP runtime then sees no GPU -- the DeviceArray test above covers it.)"""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no torch CUDA device")
    ks = "GaussianKernel(0.7,1.3,)"
    X, Y, Xm = _inputs(3000, 4, 64, 1, np.float64)
    host = ctx.sparse_fit(ks, X, Y, Xm, 0.3, 1e-4)
    Xd, Yd = torch.from_numpy(X).to("cuda:0"), torch.from_numpy(Y).to("cuda:0")
    torch.cuda.synchronize()
    dev = ctx.sparse_fit(ks, Xd, Yd, Xm, 0.3, 1e-4)
    for a, b in zip(host, dev):
        assert np.array_equal(a, b)


def _sparse_grid(count, start=-2.0, stop=5.0):
    return np.array([start + i * (stop - start) / count for i in range(count)])[:, None]


def _sparse_f(x):
    return (0.5 * np.sin(x + 10 * x) + np.sin(4 * x)) * x * x


@pytest.mark.parametrize("jitter", [0.0, 0.001])
def test_sparse_reference_core_matrix(ctx, jitter):
    """SparseInferenceTest Test2 (:135-224) on the device: inducing points = the 10 dense points on
    [-2, 5), GaussianKernel(0.23, 10), noise 0.01.  The device's Kmm^{-1} (gprx_sparse_fit) and
    cross matrix give C = Knm Kmm^{-1} Kmn ~ the dense K (the reference's bound: 1e-2 with jitter,
    2000 without), and Kmm^{-1} matches the oracle at 1e-6."""
    ks, noise = "GaussianKernel(0.23,10,)", 0.01
    X = _sparse_grid(10)
    Y = _sparse_f(X)
    Kinv, _, _ = ctx.sparse_fit(ks, X, Y, X, noise, jitter)
    Knm = ctx.cross_matrix(ks, X, X)
    K = ctx.kernel_matrix(ks, X)
    assert np.linalg.norm(Knm @ Kinv @ Knm.T - K) < (1e-2 if jitter > 0 else 2000)
    _, Ki_r, _, _, _ = O.sparse_core(ks, X, X, noise, jitter)
    assert relerr(Kinv, Ki_r) <= 1e-6
    assert np.trace(K) == 10 * 100.0  # (GetKernelMatrixTrace, Test2.2: k(x, x) = scale^2, summed exactly)


def test_sparse_reference_inversion_config(ctx):
    """SparseInferenceTest Test1's configuration (:37-133: n = 1000, m = 25, GaussianKernel(0.23, 10),
    noise 0.1, jitter 0.5) through the device sparse likelihood: log|C| (the efficient determinant's
    logarithm: the reference's product underflows here) and the value and gradient against the
    oracle's literal N x N restatement, whose Woodbury inverse the KAT pins to the direct inverse."""
    ks, noise, jitter = "GaussianKernel(0.23,10,)", 0.1, 0.5
    Xn, Xm = _sparse_grid(1000), _sparse_grid(25)
    Y = _sparse_f(Xn[:, 0]) + np.random.default_rng(0x53504731).normal(0, noise, 1000)
    v, g, ld = ctx.sparse_lml(ks, Xn, Y, Xm, noise, jitter)
    vr, gr, _, ldr = O.sparse_lml(ks, Xn, Y, Xm, noise, jitter)
    assert abs(ld - ldr) <= 1e-9 * abs(ldr)
    assert relerr(np.asarray(g), gr) <= 1e-6


def test_sparse_reference_gradient_config(ctx):
    """SparseInferenceTest Test3 (:226-336) on the device: n = 50 + it, m = 5 + it,
    GaussianKernel(0.1 + 0.02 it, 10), noise 0.2, jitter 0.01, it = 0..9: the device gradient
    against the oracle (1e-6) and against the reference's central differences of the device
    value (h = 1e-4; within 1 for sigma, 0.1 for scale)."""
    rng = np.random.default_rng(0x53504733)
    noise, jitter, h = 0.2, 0.01, 1e-4
    for it in range(10):
        sigma, scale = 0.1 + it * 0.02, 10.0
        n, m = 50 + it, 5 + it
        Xn, Xm = _sparse_grid(n), _sparse_grid(m)
        Y = _sparse_f(Xn[:, 0]) + rng.normal(0, noise, n)
        _ = rng.normal(0, noise, m)
        ks = f"GaussianKernel({sigma!r},{scale!r},)"
        _, g, _ = ctx.sparse_lml(ks, Xn, Y, Xm, noise, jitter)
        _, gr, _, _ = O.sparse_lml(ks, Xn, Y, Xm, noise, jitter)
        assert relerr(np.asarray(g), gr) <= 1e-6, it

        def val(sg, sc):
            return ctx.sparse_lml(f"GaussianKernel({sg!r},{sc!r},)", Xn, Y, Xm, noise, jitter, grad=False)[0]
        assert abs(g[0] - (val(sigma + h / 2, scale) - val(sigma - h / 2, scale)) / h) <= 1
        assert abs(g[1] - (val(sigma, scale + h / 2) - val(sigma, scale - h / 2)) / h) <= 0.1


def test_sparse_streamed_block_reuse(monkeypatch):
    """The streamed Kmn block lives in the context between fits and only the columns a longer
    chunk left behind are re-zeroed (gprx_api.cpp SparseNE::dA_zero): fits of different lengths
    (a ragged last chunk, then whole chunks, then ragged again) on one context give the same bits
    as the same fits on fresh contexts."""
    import gpr_amd
    monkeypatch.setenv("GPRX_SPARSE_CHUNK", "2048")
    ks = CASES[0][0]
    shapes = [(5000, 11), (4096, 12), (3000, 13), (5000, 11)]
    shared = gpr_amd.Context(0)
    try:
        got = []
        for n, seed in shapes:
            X, Y = make_data(n, 8, 1)
            X = X + 1e-3 * seed
            Xm = X[:: n // 300][:300].copy()
            got.append(shared.sparse_fit(ks, X, Y, Xm, 0.3, 1e-3, np.float64))
    finally:
        shared.close()
    for (n, seed), g in zip(shapes, got):
        X, Y = make_data(n, 8, 1)
        X = X + 1e-3 * seed
        Xm = X[:: n // 300][:300].copy()
        fresh = gpr_amd.Context(0)
        try:
            ref = fresh.sparse_fit(ks, X, Y, Xm, 0.3, 1e-3, np.float64)
        finally:
            fresh.close()
        for a, b in zip(g, ref):
            assert np.array_equal(a, b)
