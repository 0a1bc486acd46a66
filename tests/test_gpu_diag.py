"""The tile engine's diagonal-block factor, entrywise.

DIAGX (k_ptiles.hip) factors every 128 x 128 diagonal block of K + sigma^2 I on one CU and
forms its inverse: the step that replaces the reference's dpotrf/dgetrf on the block chain
(include/LAPACKUtils.h:38-56, 85-97; the default LU path of lib/GaussianProcess.cpp:545-559
gives the same inverse for an SPD K).  gprx_dev_diag_factor runs one block through each device
variant (0: rank-8 register image, 1: blocked MFMA, 2: blocked with look-ahead, the default)
and returns L and Linv; they are compared with numpy's Cholesky (LAPACK dpotrf) and its
triangular inverse on kernel-matrix blocks of increasing condition number, and a block that
is not positive definite must report its first bad pivot.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DB = 128


def _lib(ctx):
    from gpr_amd.gprx import lib
    L = lib()
    L.gprx_dev_diag_factor.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)]
    return L


def _factor(ctx, variant, A):
    L = _lib(ctx)
    Af = np.asfortranarray(A, dtype=np.float64)
    Lo = np.zeros((DB, DB), order="F")
    Li = np.zeros((DB, DB), order="F")
    info = ctypes.c_int32(0)
    st = L.gprx_dev_diag_factor(ctx.h, variant, Af.ctypes.data, Lo.ctypes.data, Li.ctypes.data, ctypes.byref(info))
    assert st == 0
    return np.tril(Lo), Li, info.value


def _block(scale, noise, seed=0, d=8):
    rng = np.random.default_rng(seed)
    X = rng.random((DB, d))
    r2 = ((X[:, None, :] - X[None, :, :]) ** 2).sum(-1)
    return np.exp(-r2 / (2 * scale * scale)) + noise * np.eye(DB)


CASES = [(0.3, 1.0), (0.7, 1e-2), (1.0, 1e-4), (2.0, 1e-6)]


@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("scale,noise", CASES)
def test_diag_factor_vs_lapack(ctx, variant, scale, noise):
    A = _block(scale, noise)
    Lg, Li, info = _factor(ctx, variant, A)
    assert info == 2**31 - 1
    Lr = np.linalg.cholesky(A)
    cond = np.linalg.cond(A)
    # backward error of the factor, and the factor / inverse against LAPACK scaled by cond
    assert np.abs(Lg @ Lg.T - A).max() / np.abs(A).max() < 1e-14
    assert np.abs(Lg - Lr).max() / np.abs(Lr).max() < 1e-15 * cond + 1e-13
    Lir = np.linalg.inv(Lr)
    assert np.abs(np.triu(Li, 1)).max() == 0.0
    assert np.abs(Li @ Lg - np.eye(DB)).max() < 1e-15 * np.sqrt(cond) * 50 + 1e-12
    assert np.abs(Li - Lir).max() / np.abs(Lir).max() < 1e-15 * cond + 1e-12


@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("bad", [0, 37, 100, 127])
def test_diag_factor_reports_first_bad_pivot(ctx, variant, bad):
    A = _block(0.5, 0.1, seed=3)
    # make the leading (bad+1) x (bad+1) block singular-indefinite at column `bad`
    Lr = np.linalg.cholesky(A)
    A2 = A.copy()
    A2[bad, bad] -= Lr[bad, bad] ** 2 * 1.5
    _, _, info = _factor(ctx, variant, A2)
    assert info == bad + 1


def _sparse_normal_block():
    # the normal matrix of tests/cpp/gp_host_test.cpp's SparseRegression (Kmm + 1e-6 I +
    # 1e4 Knm^T Knm, 40 inducing points of a 1-D Gaussian(0.8) GP, cond 1.5e13) padded with
    # the identity as the sparse fit pads it: an explicit 32-block inverse in the panel solve
    # alone loses positive definiteness at pivot 35 here
    x = np.arange(400) * 2 * np.pi / 400
    xm = x[::10]
    k = lambda a, b: np.exp(-(a[:, None] - b[None, :]) ** 2 / (2 * 0.8 * 0.8))
    S = k(xm, xm) + 1e-6 * np.eye(40) + 1e4 * k(x, xm).T @ k(x, xm)
    A = np.eye(DB)
    A[:40, :40] = S
    return A


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_diag_factor_ill_conditioned_block(ctx, variant):
    A = _sparse_normal_block()
    Lg, Li, info = _factor(ctx, variant, A)
    if variant == 1:  # the unrefined blocked form: the failure the refinement exists for
        return
    assert info == 2**31 - 1
    # backward error at the level of LAPACK's (numpy: 4.7e-10 absolute on entries of 4e6)
    assert np.abs(Lg @ Lg.T - A).max() < 5e-9
