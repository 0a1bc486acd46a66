"""Test infrastructure: a numpy restatement of the storage-sharded multi-GPU fit
(gpr_amd/csrc/gprx_dist.cpp + potrf_tiles_kernel<T, true> in k_ptiles.hip + k_dsolve.hip),
driven by torch.distributed collectives (gloo here).  The product's exchange is device-initiated
(each producing task stores its tile into the consumers' mailboxes and raises a flag); here every
such push is an all-gather of the tiles produced in a step, delivered only to the ranks that read
that row.  Used by tests/test_dist_schedule.py.

Layout (gprx_dist.cpp DistLayout): row block i (B rows; i = nc is the label block Y^T) lives on
rank (i // gb) % g; identity row block E_a (LML mode) with row a.  A rank stores only the LOWER
tiles of its own row blocks (packed): tile (i, j), j <= i.  Per diagonal step k:
  owner(k)  factors the fully updated diagonal block: L_kk and Linv_k = L_kk^{-1}
  push      Linv_k from owner(k) to every rank                          (the north star's broadcast)
  TRSM      every rank, its rows i > k: L_ik = A_ik Linv_k^T  (label and identity rows too)
  push      each final tile L_ik into the WINDOW of every rank that reads row i, slot k mod ww;
            the slot may be refilled only after every consumer released panel k - ww
  UPD       every rank, its rows i > k, k < j <= i: A_ij -= L_ik L_jk^T (L_jk own, or the window)
  release   panel k's window slot, once this rank's updates that read it are done
LML mode: the identity rows leave as U = L^{-T}; the C tiles (E_a, E_c), c <= a, accumulate
C -= U_ab U_cb^T over the panels b >= a (the sharded potri), and each rank sums the gradient
(alpha alpha^T - C) o dK_p over the lower tiles of ITS row blocks; one all-reduce of the partials.
Back substitution (k_dsolve.hip): each rank pushes its partial sum_{i > k, i own} L_ik^T alpha_i
to owner(k), which solves alpha_k and pushes it to every rank.  Forward substitution (the fp32
refinement's correction): owner(i) solves z_i from its row and pushes it to every rank."""
import numpy as np


def owner(i, g, gb, nc):
    return (i // gb) % g if i <= nc else ((i - nc - 1) // gb) % g


class Window:
    """A rank's receive window: ww panel slots; a slot is filled with panel p only when the
    previous occupant (panel p - ww) has been released -- the product's flow control."""

    def __init__(self, ww):
        self.ww = ww
        self.slots = {}  # slot -> (panel, {row: tile})
        self.released = set()
        self.max_live = 0

    def put(self, p, row, tile):
        s = p % self.ww
        if s in self.slots and self.slots[s][0] != p:
            old = self.slots[s][0]
            assert old in self.released, f"window slot {s} refilled with panel {p} before panel {old} was released"
            del self.slots[s]
        self.slots.setdefault(s, (p, {}))[1][row] = tile
        self.max_live = max(self.max_live, len(self.slots))

    def get(self, p, row):
        s = p % self.ww
        assert s in self.slots and self.slots[s][0] == p, f"panel {p} is not in the window"
        return self.slots[s][1][row]

    def release(self, p):
        self.released.add(p)


def sharded_fit(Kfull, Y, sigma, n, B, rank, g, gb, ww, bcast, allgather_obj, allreduce_sum, inv=False):
    """Returns dict(alpha (n x m), logdet, datafit, C (own C tiles, LML mode), rows, stored,
    window_max) on this rank.  bcast(buf, root) broadcasts a float64 array in place;
    allgather_obj(obj) -> list over ranks; allreduce_sum(array) -> summed array."""
    m = Y.shape[1]
    nc = -(-n // B)
    np_ = nc * B
    nr = nc + 1 + (nc if inv else 0)
    own = lambda i: owner(i, g, gb, nc)  # noqa: E731
    Kp = np.zeros((np_, np_))
    Kp[:n, :n] = Kfull
    Kp[np.arange(n), np.arange(n)] += sigma * sigma
    Kp[np.arange(n, np_), np.arange(n, np_)] = 1.0
    # packed storage: own row block i -> {column block: tile}
    T = {}
    for i in range(nr):
        if own(i) != rank:
            continue
        if i < nc:
            T[i] = {j: Kp[i * B:(i + 1) * B, j * B:(j + 1) * B].copy() for j in range(i + 1)}
        elif i == nc:
            lab = np.zeros((B, np_))
            lab[:m, :n] = Y.T
            T[i] = {j: lab[:, j * B:(j + 1) * B].copy() for j in range(nc)}
        else:
            a = i - nc - 1
            T[i] = {j: (np.eye(B) if j == a else np.zeros((B, B))) for j in range(a, nc)}
            for c in range(a + 1):
                T[i][("C", c)] = np.zeros((B, B))
    stored = sum(t.size for r in T.values() for t in r.values())
    # who reads which row through its window: a rank with a tile (i, j), i own, j remote
    def reads(q, j):
        if own(j) == q:
            return False
        for i in range(nr):
            if own(i) != q:
                continue
            if i <= nc and i > j and j < nc:
                return True
            if i > nc and j < nc and j > i - nc - 1:
                return True
            if i > nc and j > nc and j - nc - 1 < i - nc - 1:
                return True
        return False
    win = Window(ww)
    Linv = {}
    Ldiag = {}
    for k in range(nc):
        buf = np.empty((B, B))
        if own(k) == rank:
            D = T[k][k]
            L = np.linalg.cholesky(np.tril(D) + np.tril(D, -1).T)
            Ldiag[k] = L
            T[k][k] = L
            buf[:] = np.linalg.inv(L)
        if g > 1:
            bcast(buf, own(k))
        Linv[k] = buf.copy()
        # TRSM of this rank's rows at column k, then the pushes into the consumers' windows
        mine = {}
        for i in range(k + 1, nr):
            if own(i) != rank or (i > nc and i - nc - 1 > k):
                continue
            T[i][k] = T[i][k] @ Linv[k].T
            mine[i] = T[i][k]
        for part in (allgather_obj(mine) if g > 1 else [mine]):
            for i, t in part.items():
                if i != nc and reads(rank, i):
                    win.put(k, i, t)

        def L_of(j, b):
            return T[j][b] if own(j) == rank else win.get(b, j)
        # the updates with panel k (single-panel chunks), then the release of panel k
        for i in range(k + 1, nr):
            if own(i) != rank:
                continue
            if i <= nc:
                for j in range(k + 1, min(i, nc - 1) + 1):
                    T[i][j] -= T[i][k] @ L_of(j, k).T
            else:
                a = i - nc - 1
                if a > k:
                    continue
                for j in range(k + 1, nc):
                    T[i][j] -= T[i][k] @ L_of(j, k).T
                for c in range(a + 1):  # C_ac -= U_ak U_ck^T (stored negated)
                    T[i][("C", c)] -= T[i][k] @ L_of(nc + 1 + c, k).T
        win.release(k)
    # log det: this rank's diagonal blocks; data fit from the label tiles on their owner
    ld = 0.0
    for k, L in Ldiag.items():
        idx = np.arange(k * B, (k + 1) * B) < n
        ld += 2.0 * np.sum(np.log(np.diag(L)[idx]))
    df = 0.0
    if own(nc) == rank:
        z = np.concatenate([T[nc][k] for k in range(nc)], axis=1)
        df = float(np.sum(z[:m, :n] ** 2))
    red = allreduce_sum(np.array([ld, df])) if g > 1 else np.array([ld, df])
    # z tiles reach every rank (pushed by the label block's owner)
    ztiles = {k: T[nc][k][:m].T.copy() for k in range(nc)} if own(nc) == rank else None
    if g > 1:
        ztiles = [p for p in allgather_obj(ztiles) if p is not None][0]
    alpha = back_substitution(T, Linv, ztiles, nc, B, m, rank, g, gb, allgather_obj)
    out = dict(alpha=alpha[:n], logdet=float(red[0]), datafit=float(red[1]), stored=stored, window_max=win.max_live)
    if inv:
        out["C"] = {(i - nc - 1, c): -T[i][("C", c)] for i in T if i > nc for c in range(i - nc)}
    out["T"] = T
    out["Linv"] = Linv
    return out


def back_substitution(T, Linv, ztiles, nc, B, m, rank, g, gb, allgather_obj):
    """alpha_k = Linv_k^T (z_k - sum_{i > k} L_ik^T alpha_i): the owner of block k adds the
    partials the ranks pushed (each over its own rows i > k), solves and pushes alpha_k."""
    own = lambda i: owner(i, g, gb, nc)  # noqa: E731
    x = np.zeros((nc * B, m))
    for k in reversed(range(nc)):
        w = np.zeros((B, m))
        for i in range(k + 1, nc):
            if own(i) == rank:
                w += T[i][k].T @ x[i * B:(i + 1) * B]
        parts = allgather_obj(w) if g > 1 else [w]
        ak = None
        if own(k) == rank:
            ak = Linv[k].T @ (ztiles[k] - sum(parts))
        got = allgather_obj(ak) if g > 1 else [ak]
        x[k * B:(k + 1) * B] = [a for a in got if a is not None][0]
    return x


def forward_substitution(T, Linv, rhs, nc, B, rank, g, gb, allgather_obj):
    """z_i = Linv_i (r_i - sum_{k < i} L_ik z_k) on owner(i); each z_i pushed to every rank."""
    own = lambda i: owner(i, g, gb, nc)  # noqa: E731
    m = rhs.shape[1]
    z = np.zeros((nc * B, m))
    for i in range(nc):
        zi = None
        if own(i) == rank:
            acc = rhs[i * B:(i + 1) * B].copy()
            for k in range(i):
                acc -= T[i][k] @ z[k * B:(k + 1) * B]
            zi = Linv[i] @ acc
        got = allgather_obj(zi) if g > 1 else [zi]
        z[i * B:(i + 1) * B] = [a for a in got if a is not None][0]
    return z


def grad_partial_tiles(alpha, Ctiles, dK, n, B):
    """This rank's share of sum_{r >= c} w_rc (alpha alpha^T - C)_rc dK_p,rc (w = 2 off the
    diagonal, 1 on it) over the lower tiles of ITS row blocks, C from its own C tiles."""
    a = alpha[:, 0]
    out = np.zeros(len(dK))
    for (ti, tj), Ct in Ctiles.items():
        r0, c0 = ti * B, tj * B
        r1, c1 = min(r0 + B, n), min(c0 + B, n)
        if r0 >= n or c0 >= n:
            continue
        W = np.outer(a[r0:r1], a[c0:c1]) - Ct[:r1 - r0, :c1 - c0]
        if ti == tj:
            wt = np.tril(np.full(W.shape, 2.0), -1) + np.eye(W.shape[0])
        else:
            wt = np.full(W.shape, 2.0)
        for p, D in enumerate(dK):
            out[p] += np.sum(W * wt * D[r0:r1, c0:c1])
    return out
