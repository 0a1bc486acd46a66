"""Host-side checks of the tile-dataflow factorisation schedule (k_ptiles.hip make_schedule,
exported as gprx_dev_schedule): every task's producers hold earlier tickets (the deadlock-freedom
argument of the persistent kernel), task counts match the tile decomposition, and the simulated
makespan behaves.  No device needed."""
import ctypes

import numpy as np
import os

import pytest

from gpr_amd.gprx import lib


def _sched(nc, nr, P=256, build=False, ident=False, ratio=0, pair=0):
    """ratio: the chunk rule (0 = the fixed rule, r > 0 = width capped at r x the panels left,
    None = the rule the simulated makespan picks); pair: paired updates from row j + pair (0 =
    none, None = the f64 default, k_ptiles.hip default_pair)."""
    L = lib()
    L.gprx_dev_schedule.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]
    est = ctypes.c_double()
    n = ctypes.c_int64()
    sel = (0 if ratio is None else (ratio + 1) << 8) | (0 if pair is None else (pair + 1) << 16)
    st = L.gprx_dev_schedule(nc, nr, P, (1 if build else 0) | (2 if ident else 0) | sel, ctypes.byref(est),
                             ctypes.byref(n))
    return st, n.value, est.value


W_DEF = 64  # k_ptiles.hip Params defaults: update chunk width, single-panel tail by size


NPARTS = 8  # TPART tasks per split step of the f64 schedule (k_ptiles.hip tp_parts)


def tparts(nc):
    """The split diagonal step (f64 schedule): TPART(k, 0..7) for every k >= 1."""
    return NPARTS * max(0, nc - 1)


def near_def(nc):
    return 1 if nc <= 64 else 0


def _expected_tasks(nc, nr, W=W_DEF, near=None):
    """Task count of the chunking rule (k_ptiles.hip tile_chunks): W-aligned chunks up to the
    last multiple of W at or before column j, then power-of-two pieces before the last `near`
    panels, then single panels."""
    near = near_def(nc) if near is None else near
    diag = nc
    trsm = sum(1 for k in range(nc) for i in range(k + 1, nr) if not (i == k + 1 and i < nc))
    upd = 0
    for j in range(1, nc):
        for i in range(j, nr):
            e = j - 1 if i == j else j
            if e <= 0:
                continue
            hb = min(W * (j // W), e)
            hb -= hb % W
            upd += hb // W
            b, p = hb, W // 2
            while p >= 1:
                if b + p <= e - near:
                    upd += 1
                    b += p
                p //= 2
            upd += e - b
    return diag + trsm + upd + tparts(nc)


def _ratio_chunks(e, W, near, ratio):
    """k_ptiles.hip tile_chunks with ratio > 0: greedy widest power-of-two piece p <= W
    (W-aligned when p == W) ending >= near panels before e with p <= ratio x the panels left."""
    out, b = [], 0
    while b < e:
        p = W
        while p > 1:
            end = b + p
            if not (p == W and b % W) and end <= e - near and p <= ratio * (e - end):
                break
            p //= 2
        out.append((b, p))
        b += p
    return out


def _expected_tasks_ratio(nc, nr, ratio, W=W_DEF):
    near = near_def(nc)
    trsm = sum(1 for k in range(nc) for i in range(k + 1, nr) if not (i == k + 1 and i < nc))
    upd = 0
    for j in range(1, nc):
        for i in range(j, nr):
            e = j - 1 if i == j else j
            if e > 0:
                upd += len(_ratio_chunks(e, W, near, ratio))
    return nc + trsm + upd + tparts(nc)


@pytest.mark.parametrize("nc,extra", [(1, 0), (1, 1), (2, 1), (7, 1), (8, 1), (9, 1), (33, 1), (128, 1), (64, 0)])
def test_schedule_valid_and_counted(nc, extra):
    st, n, est = _sched(nc, nc + extra)
    assert st == 0, "ticket order violates a dependency"
    assert n == _expected_tasks(nc, nc + extra)
    assert est > 0


@pytest.mark.parametrize("ratio", [2, 4, 8])
@pytest.mark.parametrize("nc", [1, 9, 33, 70])
def test_schedule_ratio_rule_valid_and_counted(nc, ratio):
    """The capped chunk rule: pieces cover each tile's panels exactly once, the ticket order
    stays valid, and the count matches the restatement."""
    for e in range(1, 3 * W_DEF):
        ch = _ratio_chunks(e, W_DEF, 1, ratio)
        assert [b for b, _ in ch] == list(np.cumsum([0] + [p for _, p in ch])[:-1])
        assert sum(p for _, p in ch) == e
    st, n, est = _sched(nc, nc + 1, ratio=ratio)
    assert st == 0, "ticket order violates a dependency"
    assert n == _expected_tasks_ratio(nc, nc + 1, ratio)


def test_schedule_picks_the_shortest_rule():
    """The rule potrf_tiles uses is the candidate with the shortest simulated makespan: the
    capped rule at N = 4096 (chain-bound: DIAGX(18) waited 184 us for a 16-panel piece under the
    fixed rule); at N = 16384 the capped rule on the last column blocks only (the chain-bound
    tail), the fixed rule elsewhere (throughput-bound: fewer tasks)."""
    for nc, want in [(32, 2), (128, None)]:
        ests = {r: _sched(nc, nc + 1, build=True, ratio=r)[2] for r in (0, 8, 4, 2)}
        _, n_auto, est_auto = _sched(nc, nc + 1, build=True, ratio=None)
        assert est_auto <= min(ests.values())
        if want is not None:
            assert est_auto == ests[want]
        else:  # N = 16384: a capped rule on the last column blocks only (kTails) beats every plain rule
            assert est_auto < 0.995 * min(ests.values())
    assert _sched(32, 33, ratio=2)[2] < 0.92 * _sched(32, 33, ratio=0)[2]


@pytest.mark.parametrize("nc", [1, 2, 9, 64])
def test_schedule_with_fused_build(nc):
    """BUILD tasks (one per lower tile of the leading block) come first in creation order and
    every consumer of a tile depends on its build: still a valid ticket order."""
    st, n, est = _sched(nc, nc + 1, build=True)
    assert st == 0, "ticket order violates a dependency"
    assert n == _expected_tasks(nc, nc + 1) + nc * (nc + 1) // 2
    _, _, est0 = _sched(nc, nc + 1)
    assert est >= est0  # the builds add work


@pytest.mark.parametrize("nc,extra", [(1, 1), (3, 1), (9, 1), (40, 1)])
def test_schedule_with_identity_rows(nc, extra):
    """The inverse riding along (k_ptiles.hip make_schedule ni > 0): identity row block a
    gets TRSM(., k) only for k >= a and updates only from panel a on; the ticket order still
    respects every dependency, and the extra tasks match that count."""
    nr = nc + extra + nc
    st, n, est = _sched(nc, nr, build=False, ident=True)
    assert st == 0, "ticket order violates a dependency"
    W, near = W_DEF, near_def(nc)
    extra_tasks = 0
    for a in range(nc):
        extra_tasks += nc - a  # TRSM(nr0 + a, k) for k = a .. nc - 1
        for j in range(a + 1, nc):
            e = j - a
            hb = min(W * ((j - a) // W), e)
            hb -= hb % W
            cnt = hb // W
            b, p = hb, W // 2
            while p >= 1:
                if b + p <= e - near:
                    cnt += 1
                    b += p
                p //= 2
            extra_tasks += cnt + (e - b)
    assert n == _expected_tasks(nc, nc + extra) + extra_tasks


def test_schedule_makespan_scales():
    _, _, e1 = _sched(64, 65)
    _, _, e2 = _sched(128, 129)
    # 8x the flops on the same workers; the smaller size is bound by the diagonal-block chain,
    # so the simulated time grows by less than 8x but clearly more than the chain's 2x
    assert 2.2 * e1 < e2 < 10.0 * e1


def test_schedule_more_workers_never_slower():
    _, _, e64 = _sched(96, 97, P=64)
    _, _, e256 = _sched(96, 97, P=256)
    assert e256 <= e64


def _dist_sched(nc, P, g, gb, ww, build=True, inv=False, ratio=0):
    L = lib()
    L.gprx_dev_dist_schedule.argtypes = [ctypes.c_int32] * 6 + [ctypes.POINTER(ctypes.c_double),
                                                                 ctypes.POINTER(ctypes.c_int32),
                                                                 ctypes.POINTER(ctypes.c_int64)]
    est, w, nt = ctypes.c_double(), ctypes.c_int32(), ctypes.c_int64()
    st = L.gprx_dev_dist_schedule(nc, P, g, gb, ww, (1 if build else 0) | (2 if inv else 0) | ((ratio + 1) << 8),
                                  ctypes.byref(est), ctypes.byref(w), ctypes.byref(nt))
    return st, est.value, w.value, nt.value


def test_dist_schedule_makespan_scales_and_is_chain_bound():
    # C3 (nc = 128, one label row block) on g ranks of 256 workers, the best of the row-block
    # groupings and windows gprx_dist.cpp picks from: more ranks never simulate slower, and the
    # makespan stays above the DIAGX chain (nc diagonal steps of the cost model's 70 us) -- the
    # sharded fit is chain-bound at 8 ranks
    best = {}
    for g in (1, 2, 4, 8):
        ests = []
        for gb in (1, 2, 4, 8):
            if g > 1 and 128 < 2 * gb * g:
                continue
            for ww in ((128,) if g == 1 else (8, 16, 32, 64)):
                st, est, w, _ = _dist_sched(128, 256, g, gb, ww)
                assert st == 0 and est > 0 and 2 * w <= ww
                ests.append(est)
        best[g] = min(ests)
    assert best[2] < best[1] and best[4] < best[2] and best[8] <= best[4]
    assert best[8] > 128 * 70.0


def test_dist_schedule_window_flow_control():
    # windows down to 2 panels (single-panel chunks) still give a valid ticket order on every
    # rank (the simulation would raise on a cycle: the flow-control edges rel(q, p) -> pushes of
    # panel p + ww never close one), including the LML mode with identity rows and C tiles
    for ww in (2, 3, 4, 8):
        for g in (2, 3, 5):
            st, est, w, nt = _dist_sched(24, 30, g, 2, ww)
            assert st == 0 and est > 0 and w == max(1, 2 ** int(np.log2(max(1, ww // 2))))
            st, est, w, nt = _dist_sched(16, 30, g, 1, ww, inv=True)
            assert st == 0 and est > 0


def test_dist_schedule_capped_chunk_rule():
    # the capped update-chunk rule (gprx_dist.cpp tries ratios 4 and 2 for the chosen grouping
    # and window) keeps every rank's ticket order valid, flow control and LML mode included, and
    # shortens the chain-bound N = 4096 shape
    for ratio in (2, 4):
        for ww in (2, 4, 8):
            for g in (2, 3):
                st, est, w, nt = _dist_sched(24, 30, g, 2, ww, ratio=ratio)
                assert st == 0 and est > 0
                st, est, w, nt = _dist_sched(16, 30, g, 1, ww, inv=True, ratio=ratio)
                assert st == 0 and est > 0
    e0 = _dist_sched(32, 120, 2, 2, 16)[1]
    e2 = _dist_sched(32, 120, 2, 2, 16, ratio=2)[1]
    assert e2 < e0


def test_dist_schedule_lml_mode_costs_about_three_factorisations():
    # the inverse riding along: n^3/3 (factor) + n^3/3 (U = L^{-T}) + n^3/3 (C = U U^T) flops
    st, e1, _, _ = _dist_sched(48, 64, 2, 2, 16)
    st2, e3, _, _ = _dist_sched(48, 64, 2, 2, 16, inv=True)
    assert st == 0 and st2 == 0
    assert 1.8 * e1 < e3 < 4.0 * e1


def test_dist_schedule_rejects_bad_arguments():
    assert _dist_sched(0, 240, 1, 1, 8)[0] != 0
    assert _dist_sched(4, 240, 0, 1, 8)[0] != 0
    assert _dist_sched(4, 240, 33, 1, 8)[0] != 0


def _sched_list(nc, nr, P=256, ratio=None, ident=False):
    L = lib()
    L.gprx_dev_schedule_list.restype = ctypes.c_int64
    L.gprx_dev_schedule_list.argtypes = [ctypes.c_int32] * 4 + [ctypes.POINTER(ctypes.c_int32), ctypes.c_int64]
    flags = (2 if ident else 0) | (0 if ratio is None else (ratio + 1) << 8)
    n = L.gprx_dev_schedule_list(nc, nr, P, flags, None, 0)
    assert n > 0
    out = np.zeros((n, 4), np.int32)
    assert L.gprx_dev_schedule_list(nc, nr, P, flags, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), n) == n
    return out


@pytest.mark.parametrize("nc,ratio,ident", [(2, None, False), (9, 0, False), (33, 2, False), (40, 0, True),
                                            (128, None, False)])
def test_schedule_split_step_ticket_order(nc, ratio, ident):
    """The split diagonal step's deadlock-freedom argument (k_ptiles.hip order_tparts): the eight
    TPART(k, c) tickets come in the order c = 7, .., 0, after DIAGX(k - 1) and before DIAGX(k),
    and no other k's parts lie between them -- so at most seven workgroups ever wait on a
    sibling part and P >= 8 workers always leave one to claim the next ticket."""
    lst = _sched_list(nc, 2 * nc + 1 if ident else nc + 1, ratio=ratio, ident=ident)
    typ = lst[:, 0] & 0xFF
    diag = {int(lst[q, 1]): q for q in np.nonzero(typ == 0)[0]}
    assert sorted(diag) == list(range(nc))
    tp = np.nonzero(typ == 4)[0]
    assert len(tp) == tparts(nc)
    for k in range(1, nc):
        q = tp[lst[tp, 1] == k]
        assert list(lst[q, 2]) == list(range(NPARTS - 1, -1, -1))
        assert diag[k - 1] < q[0] and q[-1] < diag[k]
        assert np.all(lst[tp[(tp > q[0]) & (tp < q[-1])], 1] == k)


def test_schedule_split_step_needs_eight_workers():
    """With fewer workers than parts the parts could all wait on a sibling that no worker is
    left to claim: the schedule falls back to the whole diagonal step inside DIAGX."""
    lst = _sched_list(9, 10, P=NPARTS - 1, ratio=0)
    assert not np.any((lst[:, 0] & 0xFF) == 4)
    assert len(lst) == _expected_tasks(9, 10) - tparts(9)


def _sched_list_pair(nc, nr, build=True, ratio=0, pair=0, ident=False):
    """The ticket list (gprx_dev_schedule_list); pair: paired updates from row j + pair (0 none,
    None the default rule); ratio None: the simulation's chunk rule."""
    L = lib()
    L.gprx_dev_schedule_list.argtypes = [ctypes.c_int32] * 4 + [ctypes.c_void_p, ctypes.c_int64]
    L.gprx_dev_schedule_list.restype = ctypes.c_int64
    out = np.zeros((400000, 4), np.int32)
    flags = ((1 if build else 0) | (2 if ident else 0) | (0 if ratio is None else (ratio + 1) << 8)
             | (0 if pair is None else (pair + 1) << 16))
    n = L.gprx_dev_schedule_list(nc, nr, 256, flags, out.ctypes.data, out.shape[0])
    assert n > 0
    return out[:n]


@pytest.mark.parametrize("nc,pair", [(2, 1), (9, 1), (9, 2), (33, 2), (40, 4), (128, 2)])
def test_schedule_paired_updates(nc, pair):
    """Paired updates (T_UPD2, k_ptiles.hip make_schedule pair > 0): the off-diagonal tiles of
    column j from row j + pair down to the label row go in vertical pairs, each pair's (identical)
    chunks as one task; every tile's panels are still applied exactly once, in order, by tickets
    that come after the producers of their operands (replayed here), the identity rows and the
    `pair` - 1 tiles below the diagonal stay single, and the ticket order is valid."""
    nr = nc + 1
    st, n, est = _sched(nc, nr, build=True)
    assert st == 0
    L = _sched_list_pair(nc, nr, pair=pair)
    typ, nb = L[:, 0] & 0xFF, L[:, 0] >> 8
    ii, jj, b0 = L[:, 1], L[:, 2], L[:, 3]
    # per tile: the (b0, nb) chunks in ticket order
    applied = {}
    for q in np.where((typ == 2) | (typ == 5))[0]:
        rows = [ii[q]] if typ[q] == 2 else [ii[q], ii[q] + 1]
        if typ[q] == 5:
            assert ii[q] > jj[q] and ii[q] - jj[q] >= pair and (ii[q] - jj[q] - pair) % 2 == 0 and ii[q] + 1 <= nc
        for r in rows:
            applied.setdefault((r, jj[q]), []).append((int(b0[q]), int(nb[q]), int(q)))
    for (r, j), ch in applied.items():
        e = j - 1 if r == j else j
        pos = 0
        for b, k, q in ch:  # contiguous, in order, covering [0, e)
            assert b == pos, (r, j, ch)
            pos += k
        assert pos == e, (r, j, ch)
    # the pairs replace two single tasks each: fewer tickets than the unpaired schedule
    L0 = _sched_list_pair(nc, nr, pair=0)
    n_upd0 = int(((L0[:, 0] & 0xFF) == 2).sum())
    n_pairs = int((typ == 5).sum())
    assert int((typ == 2).sum()) + 2 * n_pairs == n_upd0
    if nc >= 9:
        assert n_pairs > 0
    # producers before consumers: a paired task's operand rows are final (their TRSM / DIAGX
    # tickets) for every panel of its chunk before it
    final = {}
    for q in range(len(L)):
        if typ[q] == 1:
            final[(ii[q], jj[q])] = q
        elif typ[q] == 0:
            final[(ii[q], ii[q])] = q
    for q in np.where(typ == 5)[0]:
        for b in range(b0[q], b0[q] + nb[q]):
            for r in (ii[q], ii[q] + 1, jj[q]):
                p = final.get((r, b))
                if p is None and r == b + 1:  # L_{b+1,b}: published by DIAGX(b + 1) (or its parts)
                    p = final.get((r, r))
                assert p is not None and p < q, (q, r, b)


def test_schedule_default_pairing_rule():
    """The f64 default (k_ptiles.hip default_pair: rows from j + 4, chunks of >= 4 panels, not in
    the last 32 columns) at C3's shape: a valid ticket order with paired tasks, none of them in the
    last 32 column blocks or narrower than 4 panels; at C2's shape (32 column blocks) no pairs."""
    st, n, est = _sched(128, 129, build=True, ratio=None, pair=None)
    assert st == 0 and n > 0
    L = _sched_list_pair(128, 129, ratio=None, pair=None)
    typ, nb, jj = L[:, 0] & 0xFF, L[:, 0] >> 8, L[:, 2]
    p = typ == 5
    assert p.sum() > 1000
    assert np.all(jj[p] < 128 - 32) and np.all(nb[p] >= 4)
    L2 = _sched_list_pair(32, 33, ratio=None, pair=None)
    assert not np.any((L2[:, 0] & 0xFF) == 5)


@pytest.mark.parametrize("nc,pair", [(3, 1), (9, 2), (40, 4), (65, 4)])
def test_schedule_paired_identity_rows(nc, pair):
    """The LML mode with pairs (k_ptiles.hip make_schedule ident_even): identity row blocks go
    in pairs (E_2s, E_2s+1), both updating from panel 2s -- the odd row's block at column 2s is
    the zero tile potrf_tiles stores, so it has no producer; every other tile's panels are applied
    once, in order, after their operands are final; the odd rows' TRSMs still start at their own
    block; the ticket order is valid (simulated) and has paired identity-row tasks."""
    nr = 2 * nc + 1
    nr0 = nc + 1
    st, n, est = _sched(nc, nr, build=True, ident=True, pair=pair)
    assert st == 0
    L = _sched_list_pair(nc, nr, pair=pair, ident=True)
    typ, nb = L[:, 0] & 0xFF, L[:, 0] >> 8
    ii, jj, b0 = L[:, 1], L[:, 2], L[:, 3]
    applied = {}
    for q in np.where((typ == 2) | (typ == 5))[0]:
        rows = [ii[q]] if typ[q] == 2 else [ii[q], ii[q] + 1]
        if typ[q] == 5 and ii[q] >= nr0:
            assert (ii[q] - nr0) % 2 == 0 and ii[q] + 1 < nr
        for r in rows:
            applied.setdefault((r, jj[q]), []).append((int(b0[q]), int(nb[q]), int(q)))
    start = lambda r: 0 if r < nr0 else (r - nr0) - ((r - nr0) & 1)
    for (r, j), ch in applied.items():
        e = j - 1 if r == j else j
        pos = start(r)
        for b, k, q in ch:
            assert b == pos, (r, j, ch)
            pos += k
        assert pos == e, (r, j, ch)
    for a in range(nc):  # every identity tile right of the block gets its updates
        for j in range(a + 1, nc):
            assert (nr0 + a, j) in applied
    if nc >= 9:
        assert np.any((typ == 5) & (ii >= nr0))
    trs = {(int(ii[q]), int(jj[q])) for q in np.where(typ == 1)[0]}
    for a in range(nc):
        assert {k for (r, k) in trs if r == nr0 + a} == set(range(a, nc))
    final = {}
    for q in range(len(L)):
        if typ[q] == 1:
            final[(ii[q], jj[q])] = q
        elif typ[q] == 0:
            final[(ii[q], ii[q])] = q
    for q in np.where((typ == 5) | (typ == 2))[0]:
        rows = (ii[q], jj[q]) if typ[q] == 2 else (ii[q], ii[q] + 1, jj[q])
        for b in range(b0[q], b0[q] + nb[q]):
            for r in rows:
                if r >= nr0 and b == r - nr0 - 1 and (r - nr0) % 2 == 1:
                    continue  # the zero tile (E_2s+1, 2s)
                if r < nc and b == r:
                    continue  # a diagonal tile's own panel is never an operand
                p = final.get((r, b))
                if p is None and r == b + 1:
                    p = final.get((r, r))
                assert p is not None and p < q, (q, r, b)
