"""Independent cross-check of the CPU oracle against numpy/scipy formulas (no shared code)."""
import numpy as np
import pytest
import scipy.linalg as sla

from oracle import oracle as O
from tests.helpers import make_data, make_queries, relerr


def np_leaf(name, p, A, B):
    diff = A[:, None, :] - B[None, :, :]
    r2 = np.sum(diff ** 2, axis=-1)
    if name == "G":
        sigma, scale = p
        return scale ** 2 * np.exp(-0.5 * r2 / sigma ** 2)
    if name == "GE":
        sigma, scale = p
        return np.exp(scale) ** 2 * np.exp(-0.5 * r2 / np.exp(sigma) ** 2)
    if name == "W":
        return np.where(r2 == 0, p[0] ** 2, 0.0)
    if name == "RQ":
        scale, sigma, alpha = p
        return scale ** 2 * (1 + 0.5 * r2 / (sigma ** 2 * alpha)) ** (-alpha)
    if name == "P":
        scale, b, sigma = p
        return scale ** 2 * np.exp(-0.5 * np.sum(np.sin(b * diff) ** 2, axis=-1) / sigma ** 2)
    raise ValueError(name)


CASES = [
    ("GaussianKernel(0.7,1.3,)", lambda A, B: np_leaf("G", (0.7, 1.3), A, B)),
    ("GaussianExpKernel(-0.3,0.1,)", lambda A, B: np_leaf("GE", (-0.3, 0.1), A, B)),
    ("RationalQuadraticKernel(1.1,0.6,1.5,)", lambda A, B: np_leaf("RQ", (1.1, 0.6, 1.5), A, B)),
    ("PeriodicKernel(0.9,2.5,0.8,)", lambda A, B: np_leaf("P", (0.9, 2.5, 0.8), A, B)),
    ("SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))",
     lambda A, B: np_leaf("G", (2, 0.15), A, B) + np_leaf("P", (0.1, np.pi, 1), A, B)),
    ("ProductKernel(GaussianKernel(1.5,1,),WhiteKernel(0.3,))",
     lambda A, B: np_leaf("G", (1.5, 1), A, B) * np_leaf("W", (0.3,), A, B)),
]


@pytest.mark.parametrize("ks,ref", CASES)
def test_kernel_matrix_numpy(ks, ref):
    X, _ = make_data(60, 4)
    assert relerr(O.kernel_matrix(ks, X), ref(X, X)) < 1e-13
    Q = make_queries(17, 4)
    assert relerr(O.cross_matrix(ks, Q, X), ref(Q, X)) < 1e-13


@pytest.mark.parametrize("ks,ref", CASES)
def test_fit_predict_numpy(ks, ref):
    X, Y = make_data(80, 3, 2)
    s = 0.3
    K = ref(X, X) + s * s * np.eye(80)
    a, C = O.fit(ks, X, Y, s)
    assert relerr(a, np.linalg.solve(K, Y)) < 1e-10
    assert relerr(C, np.linalg.inv(K)) < 1e-10
    Q = make_queries(9, 3)
    assert relerr(O.predict(ks, X, a, Q), ref(Q, X) @ a) < 1e-12


def test_predict_derivative_formula():
    # D(:,c) = -X^T (Kx o alpha_c), X_i = x - x_i (lib/GaussianProcess.cpp:77-79)
    ks, ref = CASES[0]
    X, Y = make_data(50, 3, 2)
    a, _ = O.fit(ks, X, Y, 0.2)
    Q = make_queries(5, 3)
    _, D = O.predict(ks, X, a, Q, with_deriv=True)
    for t in range(5):
        kx = ref(Q[t:t + 1], X)[0]
        Xd = Q[t][None, :] - X
        for c in range(2):
            assert relerr(D[t, :, c], -Xd.T @ (kx * a[:, c])) < 1e-12


@pytest.mark.parametrize("ks,ref", CASES[:5])
def test_lml_and_gradient_numpy(ks, ref):
    X, Y = make_data(70, 2)
    s = 0.4
    K = ref(X, X) + s * s * np.eye(70)
    v, g, det, ld = O.lml(ks, X, Y, s)
    sign, logdet = np.linalg.slogdet(K)
    y = Y[:, 0]
    v_np = -0.5 * y @ np.linalg.solve(K, y) - 0.5 * logdet - 70 / 2 * np.log(2 * np.pi)
    assert abs(v - v_np) < 1e-9 * max(1, abs(v_np))
    assert abs(ld - logdet) < 1e-10 * max(1, abs(logdet))
    # gradient by central differences of the numpy LML in each parameter
    node = __import__("gpr_amd").parse_kernel(ks)
    P = np.array(node.parameters())
    h = 1e-6

    def lml_np(params):
        Kp = np.zeros((70, 70))
        Kp[:] = O.kernel_matrix(_with_params(ks, params), X) + s * s * np.eye(70)
        c, low = sla.cho_factor(Kp)
        return -0.5 * y @ sla.cho_solve((c, low), y) - np.sum(np.log(np.diag(c)))

    for p in range(len(P)):
        Pp, Pm = P.copy(), P.copy()
        Pp[p] += h
        Pm[p] -= h
        fd = (lml_np(Pp) - lml_np(Pm)) / (2 * h)
        assert abs(fd - g[p]) < 1e-5 * max(1, abs(fd)), (p, fd, g[p])


def _with_params(ks, params):
    import gpr_amd
    node = gpr_amd.parse_kernel(ks)
    it = iter(params)

    def walk(n):
        if n.is_leaf:
            n.params = [float(next(it)) for _ in n.params]
        else:
            walk(n.k1)
            walk(n.k2)

    walk(node)
    return node.to_string()


def test_long_double_determinant_narrowing():
    # Likelihood.h:77-79 narrows det to T; beyond ~1e308 it becomes inf -> clamp to
    # -0.5 log(LDBL_MAX) (:183-184).  Build a case with log det > 709.
    n = 400
    X = np.arange(n, dtype=float)[:, None] * 100.0  # far apart: K ~ (s^2 + sigma_n^2) I
    Y = np.ones((n, 1))
    v, _, det, ld = O.lml("GaussianKernel(1,10,)", X, Y, 1.0, with_grad=False)
    assert ld > 709
    cp = -0.5 * np.log(np.finfo(np.longdouble).max)
    v_expected = -0.5 * np.sum(1 / 101.0 * Y[:, 0] ** 2) + cp - n / 2 * np.log(2 * np.pi)
    assert abs(v - v_expected) < 1e-6 * abs(v_expected)


def test_sparse_fit_numpy():
    ks, ref = CASES[0]
    X, Y = make_data(120, 3)
    Xm = X[::6]
    s, jit = 0.2, 1e-4
    Kinv, RV, RM = O.sparse_fit(ks, X, Y, Xm, s, jit)
    Kmm = ref(Xm, Xm) + jit * np.eye(len(Xm))
    Knm = ref(X, Xm)
    S = Kmm + Knm.T @ Knm / s ** 2
    Sig = np.linalg.inv(S)
    assert relerr(Kinv, np.linalg.inv(Kmm)) < 1e-8
    assert relerr(RV, Sig @ Knm.T @ Y / s ** 2) < 1e-6
    assert relerr(RM, Sig) < 1e-6


@pytest.mark.parametrize("ks,ref", [CASES[0], CASES[4], CASES[2]])
def test_sparse_lml_numpy(ks, ref):
    """The oracle's literal SparseGaussianLogLikelihood (include/SparseLikelihood.h:231-344)
    against an independent numpy evaluation of the Nystrom likelihood
    log N(y | 0, sigma^2 I + Knm Kmm^-1 Kmn) (dense solve, slogdet) and central differences of
    it in every kernel parameter (the reference differentiates the kernel parameters only)."""
    n, M, s, jit = 150, 15, 0.4, 1e-3
    X, Y = make_data(n, 3)
    Xm = X[:: n // M][:M].copy()
    y = Y[:, 0]
    v, g, det, ld = O.sparse_lml(ks, X, y, Xm, s, jit)

    def lml_np(kstr):
        Kmm = O.kernel_matrix(kstr, Xm) + jit * np.eye(M)
        Knm = O.cross_matrix(kstr, X, Xm)
        C = s * s * np.eye(n) + Knm @ np.linalg.solve(Kmm, Knm.T)
        sign, lgd = np.linalg.slogdet(C)
        return -0.5 * y @ np.linalg.solve(C, y) - 0.5 * lgd - n / 2 * np.log(2 * np.pi), lgd

    v_np, ld_np = lml_np(ks)
    assert abs(v - v_np) < 1e-8 * max(1, abs(v_np))
    assert abs(ld - ld_np) < 1e-8 * max(1, abs(ld_np))
    P = np.array(__import__("gpr_amd").parse_kernel(ks).parameters())
    for p in range(len(P)):
        h = 1e-5 * max(1.0, abs(P[p]))
        Pp, Pm = P.copy(), P.copy()
        Pp[p] += h
        Pm[p] -= h
        fd = (lml_np(_with_params(ks, Pp))[0] - lml_np(_with_params(ks, Pm))[0]) / (2 * h)
        assert abs(fd - g[p]) < 1e-5 * max(1, abs(fd)), (p, fd, g[p])
