"""TEST INFRASTRUCTURE — ctypes front-end of the CPU oracle (oracle/gpr_oracle.cpp).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module.  It is the parity *checker*: a restatement of the reference (agiger/GPR) GP path
on the CPU; the product (libgprx, gpr_amd/) never calls it.  See gpr_oracle.cpp for the
reference file:line each entry point restates.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

FULL_PIVOT_LU = 0
SELF_ADJOINT_EIGEN_SOLVER = 3


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        _LIB = ctypes.CDLL(path)
        _LIB.orc_last_error.restype = ctypes.c_char_p
        _LIB.orc_lapack_name.restype = ctypes.c_char_p
    return _LIB


class OracleError(RuntimeError):
    pass


def _dt(dtype):
    dtype = np.dtype(dtype)
    if dtype == np.float64:
        return "f64", ctypes.c_double
    if dtype == np.float32:
        return "f32", ctypes.c_float
    raise TypeError(dtype)


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def _call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise OracleError(lib().orc_last_error().decode())


def lapack_name():
    return lib().orc_lapack_name().decode()


def num_threads():
    return lib().orc_num_threads()


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def kernel_nparams(kstr, dtype=np.float64):
    suf, _ = _dt(dtype)
    n = ctypes.c_int()
    _call(f"orc_kernel_nparams_{suf}", kstr.encode(), ctypes.byref(n))
    return n.value


def kernel_eval(kstr, x, y, dtype=np.float64, with_grad=True):
    suf, ct = _dt(dtype)
    x, y = _c(x, dtype), _c(y, dtype)
    val = np.zeros(1, dtype)
    g = np.zeros(kernel_nparams(kstr, dtype), dtype) if with_grad else None
    _call(f"orc_kernel_eval_{suf}", kstr.encode(), _p(x), _p(y), len(x), _p(val), _p(g))
    return (val[0], g) if with_grad else val[0]


def kernel_eval_params(kstr, params, x, y, dtype=np.float64, with_grad=True):
    """Evaluate the kernel structure `kstr` for B parameter vectors (B x P) on one pair."""
    suf, _ = _dt(dtype)
    params = _c(np.atleast_2d(params), dtype)
    x, y = _c(x, dtype), _c(y, dtype)
    B = params.shape[0]
    val = np.empty(B, dtype)
    g = np.empty_like(params) if with_grad else None
    _call(f"orc_kernel_eval_params_{suf}", kstr.encode(), _p(params), B, _p(x), _p(y), len(x), _p(val), _p(g))
    return (val, g) if with_grad else val


def kernel_matrix(kstr, X, dtype=np.float64):
    suf, _ = _dt(dtype)
    X = _c(X, dtype)
    n, d = X.shape
    K = np.empty((n, n), dtype)
    _call(f"orc_kernel_matrix_{suf}", kstr.encode(), _p(X), n, d, _p(K))
    return K


def cross_matrix(kstr, A, B, dtype=np.float64):
    suf, _ = _dt(dtype)
    A, B = _c(A, dtype), _c(B, dtype)
    K = np.empty((A.shape[0], B.shape[0]), dtype)
    _call(f"orc_cross_matrix_{suf}", kstr.encode(), _p(A), A.shape[0], _p(B), B.shape[0], A.shape[1], _p(K))
    return K


def deriv_matrix(kstr, X, dtype=np.float64):
    suf, _ = _dt(dtype)
    X = _c(X, dtype)
    n, d = X.shape
    P = kernel_nparams(kstr, dtype)
    D = np.empty((P * n, n), dtype)
    _call(f"orc_deriv_matrix_{suf}", kstr.encode(), _p(X), n, d, _p(D))
    return D.reshape(P, n, n)


def invert(K, method=FULL_PIVOT_LU, stable=False):
    suf, _ = _dt(K.dtype)
    K = np.ascontiguousarray(K)
    C = np.empty_like(K)
    _call(f"orc_invert_{suf}", _p(K), K.shape[0], method, int(stable), _p(C))
    return C


def fit(kstr, X, Y, sigma, dtype=np.float64, method=FULL_PIVOT_LU, want_core=True):
    """GaussianProcess::Initialize -> (alpha = C Y, C)."""
    suf, ct = _dt(dtype)
    X, Y = _c(X, dtype), _c(Y, dtype)
    if Y.ndim == 1:
        Y = Y[:, None]
    n, d = X.shape
    m = Y.shape[1]
    alpha = np.empty((n, m), dtype)
    C = np.empty((n, n), dtype) if want_core else None
    _call(f"orc_fit_{suf}", kstr.encode(), _p(X), _p(Y), n, d, m, ct(sigma), method, _p(alpha), _p(C))
    return alpha, C


def predict(kstr, X, alpha, Xq, dtype=np.float64, with_deriv=False):
    suf, _ = _dt(dtype)
    X, alpha, Xq = _c(X, dtype), _c(alpha, dtype), _c(Xq, dtype)
    n, d = X.shape
    m = alpha.shape[1]
    q = Xq.shape[0]
    mean = np.empty((q, m), dtype)
    D = np.empty((q, d, m), dtype) if with_deriv else None
    _call(f"orc_predict_{suf}", kstr.encode(), _p(X), n, d, m, _p(alpha), _p(Xq), q, _p(mean), _p(D))
    return (mean, D) if with_deriv else mean


def posterior_cov(kstr, X, C, Xa, Xb, dtype=np.float64):
    suf, _ = _dt(dtype)
    X, C, Xa, Xb = (_c(a, dtype) for a in (X, C, Xa, Xb))
    n, d = X.shape
    out = np.empty(Xa.shape[0], dtype)
    _call(f"orc_posterior_cov_{suf}", kstr.encode(), _p(X), n, d, _p(C), _p(Xa), _p(Xb), Xa.shape[0], _p(out))
    return out


def lml(kstr, X, Y, sigma, dtype=np.float64, method=FULL_PIVOT_LU, with_grad=True):
    """GaussianLogLikelihood value (+ gradient).  Returns (value, grad, det, logdet)."""
    suf, ct = _dt(dtype)
    X, Y = _c(X, dtype), _c(Y, dtype).reshape(-1)
    n, d = X.shape
    val = np.zeros(1, dtype)
    g = np.zeros(kernel_nparams(kstr, dtype), dtype) if with_grad else None
    det = ctypes.c_double()
    ld = ctypes.c_double()
    _call(f"orc_lml_{suf}", kstr.encode(), _p(X), _p(Y), n, d, ct(sigma), method, _p(val), _p(g),
          ctypes.byref(det), ctypes.byref(ld))
    return val[0], g, det.value, ld.value


def sparse_fit(kstr, X, Y, Xm, sigma, jitter, dtype=np.float64):
    """SparseGaussianProcess::PreComputeRegression -> (Kinv, RV, RM) (no N x N core)."""
    suf, ct = _dt(dtype)
    X, Y, Xm = _c(X, dtype), _c(Y, dtype), _c(Xm, dtype)
    if Y.ndim == 1:
        Y = Y[:, None]
    n, d = X.shape
    m = Y.shape[1]
    M = Xm.shape[0]
    Kinv = np.empty((M, M), dtype)
    RV = np.empty((M, m), dtype)
    RM = np.empty((M, M), dtype)
    _call(f"orc_sparse_fit_{suf}", kstr.encode(), _p(X), _p(Y), n, d, m, _p(Xm), M, ct(sigma), ct(jitter),
          _p(Kinv), _p(RV), _p(RM))
    return Kinv, RV, RM


def sparse_core(kstr, X, Xm, sigma, jitter, dtype=np.float64):
    """The sparse likelihood's core quantities (SparseLikelihood::GetCoreMatrices,
    EfficientInversion, EfficientDeterminant; include/SparseLikelihood.h:62-145):
    returns (K = Kmm + jitter I, Kinv, Knm, Cinv = inv(sigma^2 I + Knm Kinv Knm^T) by Woodbury,
    det_eff = the long-double efficient determinant narrowed to double)."""
    suf, ct = _dt(dtype)
    X, Xm = _c(X, dtype), _c(Xm, dtype)
    n, d = X.shape
    M = Xm.shape[0]
    K, Kinv = np.empty((M, M), dtype), np.empty((M, M), dtype)
    Knm, Cinv = np.empty((n, M), dtype), np.empty((n, n), dtype)
    det = ctypes.c_double()
    _call(f"orc_sparse_core_{suf}", kstr.encode(), _p(X), n, d, _p(Xm), M, ct(sigma), ct(jitter), _p(K), _p(Kinv),
          _p(Knm), _p(Cinv), ctypes.byref(det))
    return K, Kinv, Knm, Cinv, det.value


def sparse_lml(kstr, X, Y, Xm, sigma, jitter, dtype=np.float64, with_grad=True):
    """SparseGaussianLogLikelihood value (+ gradient), N x N restatement (small n).
    Returns (value, grad, det, logdet)."""
    suf, ct = _dt(dtype)
    X, Y, Xm = _c(X, dtype), _c(Y, dtype).reshape(-1), _c(Xm, dtype)
    n, d = X.shape
    val = np.zeros(1, dtype)
    g = np.zeros(kernel_nparams(kstr, dtype), dtype) if with_grad else None
    det = ctypes.c_double()
    ld = ctypes.c_double()
    _call(f"orc_sparse_lml_{suf}", kstr.encode(), _p(X), _p(Y), n, d, _p(Xm), Xm.shape[0], ct(sigma), ct(jitter),
          _p(val), _p(g), ctypes.byref(det), ctypes.byref(ld))
    return val[0], g, det.value, ld.value
