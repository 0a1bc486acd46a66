"""Test infrastructure: a numpy restatement of the multi-GPU factorisation schedule of
gpr_amd/csrc/k_potrf.hip::potrf_dist and the sharded build of gprx_api.cpp::model_fit,
driven by torch.distributed collectives (gloo here; the product path issues the same
broadcast/all-reduce sequence through RCCL).

Per panel K (NBO columns, owner K mod W): the owner factors its fully updated panel
(diagonal block Cholesky + trsm of the rows below, including the label rows), broadcasts
the packed rows c0.. of the panel, every rank unpacks it into its full-size matrix and
updates the later panels it owns, the next panel first.  Each rank builds only its own
panels.  Used by tests/test_dist_schedule.py (world_size 2, CPU)."""
import numpy as np


def build_owned(Kfull, Y, sigma, n, np_, ld, NBO, rank, world):
    """The sharded build: rank-owned column panels of the lower triangle + noise/padding
    diagonal + label rows; everything else left zero (filled by the broadcasts)."""
    A = np.zeros((ld, np_))
    m = Y.shape[1]
    for K in range(rank, np_ // NBO, world):
        c0 = K * NBO
        for j in range(c0, c0 + NBO):
            if j < n:
                A[j:n, j] = Kfull[j:n, j]
                A[j, j] += sigma * sigma
                A[np_:np_ + m, j] = Y[j]
            else:
                A[j, j] = 1.0
    return A


def potrf_dist(A, np_, NBO, rank, world, bcast):
    """bcast(buf, root) broadcasts a float64 numpy array in place."""
    ld = A.shape[0]
    nK = np_ // NBO
    owner = lambda K: K % world  # noqa: E731
    for K in range(nK):
        c0 = K * NBO
        root = owner(K)
        pack = np.empty((ld - c0, NBO))
        if root == rank:
            # potrf_panel: factor the diagonal block, trsm every row below (label rows too)
            D = A[c0:c0 + NBO, c0:c0 + NBO]
            L = np.linalg.cholesky(np.tril(D) + np.tril(D, -1).T)
            A[c0:c0 + NBO, c0:c0 + NBO] = L
            A[c0 + NBO:, c0:c0 + NBO] = np.linalg.solve(L, A[c0 + NBO:, c0:c0 + NBO].T).T
            pack[:] = A[c0:, c0:c0 + NBO]
        if world > 1:
            bcast(pack, root)
            if root != rank:
                A[c0:, c0:c0 + NBO] = pack
        if K == nK - 1:
            break
        P = A[:, c0:c0 + NBO]
        for J in range(K + 1, nK):
            if owner(J) != rank:
                continue
            cj = J * NBO
            A[cj:, cj:cj + NBO] -= P[cj:] @ P[cj:cj + NBO].T
    return A
