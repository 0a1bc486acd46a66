"""Test infrastructure: a numpy restatement of the storage-sharded multi-GPU fit
(gpr_amd/csrc/gprx_dist.cpp + potrf_tiles_kernel<T, true> in k_ptiles.hip) and of the
distributed LML gradient reduction, driven by torch.distributed collectives (gloo here; the
product issues the same steps through RCCL).  Used by tests/test_dist_schedule.py.

Layout (gprx_dist.cpp DistLayout): row block i (B rows; i = nc is the label block, Y^T) lives
on rank (i // gb) % g; a rank stores only its own row blocks.  Per diagonal step k:
  owner(k)  factors the fully updated diagonal block: L_kk and Linv_k = L_kk^{-1}
  bcast(k)  Linv_k from owner(k) to every rank                          (ncclBroadcast)
  TRSM      every rank, its rows i > k: L_ik = A_ik Linv_k^T  (label rows too)
  panel(k)  every rank's final tiles L_ik to every other rank  (grouped ncclSend/ncclRecv)
  UPD       every rank, its rows i > k, k < j <= i: A_ij -= L_ik L_jk^T (L_jk local or received)
Then every rank holds every off-diagonal tile and every Linv_k: log det = sum over the ranks
of their diagonal blocks' 2 sum log L_ii (all-reduce), alpha by back substitution from the
tiles on each rank.

LML gradient on a distributed context (gprx_api.cpp model_lml): every rank assembles L from
its tiles, forms C = (K + s^2 I)^{-1} = L^{-T} L^{-1} (replicated), and sums
(alpha alpha^T - C) o dK_p over the lower-triangle tiles of ITS row blocks (weight 2 off the
diagonal); one all-reduce of the P partials gives delta_p = 1/2 tr((alpha alpha^T - C) D_p)
(include/Likelihood.h:204-229)."""
import numpy as np


def owner(i, g, gb):
    return (i // gb) % g


def sharded_fit(Kfull, Y, sigma, n, B, rank, g, gb, bcast, allgather_obj, allreduce_sum):
    """Returns (alpha (n x m), logdet, datafit, tiles, Linv, np_) on this rank.
    bcast(buf, root) broadcasts a float64 array in place; allgather_obj(obj) -> list over
    ranks; allreduce_sum(array) -> summed array."""
    m = Y.shape[1]
    nc = -(-n // B)
    np_ = nc * B
    own = lambda i: owner(i, g, gb)  # noqa: E731
    # the sharded build: this rank's row blocks of the lower triangle, noise on the diagonal,
    # identity on the padding; the label block holds Y^T (m rows)
    Kp = np.zeros((np_, np_))
    Kp[:n, :n] = Kfull
    Kp[np.arange(n), np.arange(n)] += sigma * sigma
    Kp[np.arange(n, np_), np.arange(n, np_)] = 1.0
    A = {}
    for i in range(nc + 1):
        if own(i) != rank:
            continue
        if i < nc:
            A[i] = np.tril(Kp[i * B:(i + 1) * B, :], i * B)  # columns <= the global row
        else:
            A[i] = np.zeros((m, np_))
            A[i][:, :n] = Y.T
    tiles, Linv, Ldiag = {}, {}, {}
    for k in range(nc):
        cs = slice(k * B, (k + 1) * B)
        buf = np.empty((B, B))
        if own(k) == rank:
            D = A[k][:, cs]
            L = np.linalg.cholesky(np.tril(D) + np.tril(D, -1).T)
            Ldiag[k] = L
            buf[:] = np.linalg.inv(L)
        if g > 1:
            bcast(buf, own(k))
        Linv[k] = buf.copy()
        mine = {}
        for i in range(k + 1, nc + 1):
            if own(i) == rank:
                A[i][:, cs] = A[i][:, cs] @ Linv[k].T
                mine[i] = A[i][:, cs].copy()
        for part in (allgather_obj(mine) if g > 1 else [mine]):
            for i, t in part.items():
                tiles[(i, k)] = t
        for i in range(k + 1, nc + 1):
            if own(i) != rank:
                continue
            for j in range(k + 1, min(i, nc - 1) + 1):
                A[i][:, j * B:(j + 1) * B] -= tiles[(i, k)] @ tiles[(j, k)].T
    # log det: this rank's diagonal blocks, then the all-reduce
    ld = 0.0
    for k, L in Ldiag.items():
        idx = np.arange(k * B, (k + 1) * B) < n
        ld += 2.0 * np.sum(np.log(np.diag(L)[idx]))
    logdet = float(allreduce_sum(np.array([ld]))[0]) if g > 1 else ld
    # alpha = L^{-T} z from the tiles (every rank), z = the label block's tiles
    z = np.concatenate([tiles[(nc, k)] for k in range(nc)], axis=1)  # m x np
    datafit = float(np.sum(z[:, :n] ** 2))
    x = np.zeros((np_, m))
    for k in reversed(range(nc)):
        r = z[:, k * B:(k + 1) * B].T.copy()
        for i in range(k + 1, nc):
            r -= tiles[(i, k)].T @ x[i * B:(i + 1) * B]
        x[k * B:(k + 1) * B] = Linv[k].T @ r
    return x[:n], logdet, datafit, tiles, Linv, np_


def assemble_L(tiles, Linv, nc, B):
    """The dense factor every rank can form from its tiles (gprx_api.cpp, distributed LML)."""
    np_ = nc * B
    L = np.zeros((np_, np_))
    for k in range(nc):
        L[k * B:(k + 1) * B, k * B:(k + 1) * B] = np.linalg.inv(Linv[k])
        for i in range(k + 1, nc):
            L[i * B:(i + 1) * B, k * B:(k + 1) * B] = tiles[(i, k)]
    return L


def grad_partial(alpha, C, dK, n, B, rank, g, gb):
    """This rank's share of sum_{r >= c} w_rc (alpha alpha^T - C)_rc dK_p,rc (w = 2 off the
    diagonal, 1 on it) over its row blocks; 1/2 of the all-reduced sum is the gradient."""
    a = alpha[:, 0]
    W = np.outer(a, a) - C[:n, :n]
    wt = np.tril(np.full((n, n), 2.0), -1) + np.eye(n)
    rows = np.zeros(n, bool)
    nc = -(-n // B)
    for i in range(nc):
        if owner(i, g, gb) == rank:
            rows[i * B:min((i + 1) * B, n)] = True
    return np.array([np.sum((W * wt * D)[rows]) for D in dK])
