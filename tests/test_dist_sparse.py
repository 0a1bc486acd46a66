"""World-size-2 gloo restatement of the row-sharded sparse fit (gprx_api.cpp sparse_fit_impl
on an RCCL context, SURVEY.md 8(e) "Sparse fit: shard N rows; per GPU accumulate Knm^T Knm
and Knm^T Y; all-reduce"): each rank forms sigma^-2 [Kmn; Y^T][Kmn; Y^T]^T over its own dense
rows, one all-reduce sums them, and every rank solves S = Kmm + jitter I + sum for RV and
RM = S^{-1}.  Checked against the oracle's restatement of the reference's single-process
PreComputeRegression (include/SparseGaussianProcess.h:274-313)."""
import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


KS = "GaussianKernel(0.7,1.3,)"


def _inputs(n, d, M):
    from gpr_amd.synth import make_data
    X, Y = make_data(n, d, 1)
    return X, Y, X[:: n // M][:M].copy()


def _worker(rank, world, port, n, d, M, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    from oracle import oracle as O
    X, Y, Xm = _inputs(n, d, M)
    lo, hi = (n * rank) // world, (n * (rank + 1)) // world  # this rank's dense rows
    Kmn = O.cross_matrix(KS, Xm, X[lo:hi])
    sigma, jitter = 0.3, 1e-4
    part = np.concatenate([Kmn, Y[lo:hi].T], axis=0)
    P = torch.from_numpy(part @ part.T / sigma ** 2)
    dist.all_reduce(P)
    P = P.numpy()
    S = O.kernel_matrix(KS, Xm) + jitter * np.eye(M) + P[:M, :M]
    RV = np.linalg.solve(S, P[:M, M:])
    RM = np.linalg.inv(S)
    np.savez(out + f"_{rank}.npz", RV=RV, RM=RM)
    dist.barrier()
    dist.destroy_process_group()


def test_row_sharded_sparse_world2(tmp_path):
    world, n, d, M = 2, 900, 3, 45
    out = str(tmp_path / "sp")
    mp.spawn(_worker, args=(world, _free_port(), n, d, M, out), nprocs=world, join=True)
    from oracle import oracle as O
    X, Y, Xm = _inputs(n, d, M)
    _, RV_r, RM_r = O.sparse_fit(KS, X, Y, Xm, 0.3, 1e-4)
    for r in range(world):
        z = np.load(out + f"_{r}.npz")
        # normwise 1e-5: the reference's Kinv (K Sigma Knm^T Y) route and the S^{-1} route differ
        # by cond(S) eps (the same bar as tests/test_gpu_sparse.py)
        assert np.max(np.abs(z["RV"] - RV_r)) <= 1e-5 * np.max(np.abs(RV_r))
        assert np.max(np.abs(z["RM"] - RM_r)) <= 1e-5 * np.max(np.abs(RM_r))


def _lml_worker(rank, world, port, n, d, M, out):
    """Row-sharded sparse likelihood (gprx_api.cpp sparse_lml_impl on an RCCL context): the
    normal equations all-reduced as in the fit, then each rank's data terms (y^T y, N) and its
    rows' gradient partials sum_{i in rank} sum_a Omega_ia dk(x_i, xm_a)/dp all-reduced once;
    the M x M part (replicated) is added after the reduction."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    from oracle import oracle as O
    X, Y, Xm = _inputs(n, d, M)
    y = Y[:, 0]
    lo, hi = (n * rank) // world, (n * (rank + 1)) // world
    sigma, jitter = 0.3, 1e-3
    s2 = sigma * sigma
    Kc = O.cross_matrix(KS, X[lo:hi], Xm)  # this rank's rows of Knm
    part = np.concatenate([Kc.T, Y[lo:hi].T], axis=0)
    P = torch.from_numpy(part @ part.T / s2)
    dist.all_reduce(P)
    P = P.numpy()
    Kmm = O.kernel_matrix(KS, Xm) + jitter * np.eye(M)
    B = Kmm + P[:M, :M]
    b = P[:M, M]
    Sig = np.linalg.inv(B)
    u = Sig @ b
    # per-rank gradient partials of the N x M part (GaussianKernel(sigma, scale): dk/dsigma,
    # dk/dscale) with Omega = sigma^-2 [(y - Kc u) u^T - Kc Sigma]
    sg, sc = 0.7, 1.3
    r2 = ((X[lo:hi, None, :] - Xm[None, :, :]) ** 2).sum(-1)
    e = np.exp(-0.5 * r2 / sg ** 2)
    D = [sc * sc * r2 / sg ** 3 * e, 2 * sc * e]
    Om = (np.outer(y[lo:hi] - Kc @ u, u) - Kc @ Sig) / s2
    loc = torch.tensor([(D[0] * Om).sum(), (D[1] * Om).sum(), y[lo:hi] @ y[lo:hi], float(hi - lo)],
                       dtype=torch.float64)
    dist.all_reduce(loc)
    gx0, gx1, yty, nn = loc.tolist()
    r2m = ((Xm[:, None, :] - Xm[None, :, :]) ** 2).sum(-1)
    em = np.exp(-0.5 * r2m / sg ** 2)
    E = [sc * sc * r2m / sg ** 3 * em, 2 * sc * em]
    W = np.outer(u, u) - (np.linalg.inv(Kmm) - Sig)
    g = np.array([gx0 - 0.5 * (W * E[0]).sum(), gx1 - 0.5 * (W * E[1]).sum()])
    ld = nn * np.log(s2) + np.linalg.slogdet(B)[1] - np.linalg.slogdet(Kmm)[1]
    v = -0.5 * (yty / s2 - b @ u) - 0.5 * ld - nn / 2 * np.log(2 * np.pi)
    np.savez(out + f"_{rank}.npz", v=v, g=g)
    dist.barrier()
    dist.destroy_process_group()


def test_row_sharded_sparse_lml_world2(tmp_path):
    world, n, d, M = 2, 700, 3, 35
    out = str(tmp_path / "spl")
    mp.spawn(_lml_worker, args=(world, _free_port(), n, d, M, out), nprocs=world, join=True)
    from oracle import oracle as O
    X, Y, Xm = _inputs(n, d, M)
    v_r, g_r, _, _ = O.sparse_lml(KS, X, Y[:, 0], Xm, 0.3, 1e-3)
    for r in range(world):
        z = np.load(out + f"_{r}.npz")
        assert abs(float(z["v"]) - v_r) <= 1e-8 * abs(v_r)
        assert np.max(np.abs(z["g"] - g_r)) <= 1e-6 * np.max(np.abs(g_r))
