"""Python model of the tile-dataflow Cholesky schedule (k_ptiles.hip make_schedule) for
exploring chunking rules and cost changes.  Unlike the C++ list scheduler it models the early
publication of L_{k,k-1} inside DIAGX(k) (k_ptiles.hip: publish(lcnt+k, k) after the trsm
phase), so chain estimates are closer to the device.

  python scripts/sched_sim.py [--nc 128] [--rule w8|geo|...] [--P 256] [cost overrides]
"""
import argparse
import heapq

DIAGX, TRSM, UPD = 0, 1, 2


def chunks_w(i, j, W=8):
    e = j - 1 if i == j else j
    if e <= 0:
        return []
    hb = max(0, min(W * (j // W), e))
    hb -= hb % W
    out = [(b, W) for b in range(0, hb - W + 1, W)]
    out += [(b, 1) for b in range(hb, e)]
    return out


def chunks_bin(i, j, W=8, near=1, first=0):
    """`first` leading single panels, W-chunks aligned at first + k W, then the remainder
    before the last `near` panels in power-of-two pieces, then singles."""
    e = j - 1 if i == j else j
    if e <= 0:
        return []
    f = min(first, e)
    out = [(b, 1) for b in range(f)]
    hb = f + max(0, min(W * ((j - f) // W), e - f))
    hb -= (hb - f) % W
    out += [(b, W) for b in range(f, hb - W + 1, W)]
    b = hb
    lim = e - near
    p = W // 2
    while p >= 1:
        if b + p <= lim:
            out.append((b, p))
            b += p
        p //= 2
    out += [(x, 1) for x in range(b, e)]
    return out


def chunks_bounds(i, j, bounds, near=0):
    """bounds: increasing chunk start panels (global); a chunk [s, s') is used whole when
    s' <= e - near; the remaining panels are singles."""
    e = j - 1 if i == j else j
    if e <= 0:
        return []
    out = []
    b = 0
    for s, s2 in zip(bounds, bounds[1:]):
        if s2 > e - near:
            break
        if s2 - s >= 1:
            out.append((s, s2 - s))
        b = s2
    out += [(x, 1) for x in range(b, e)]
    return out


def build(nc, nr, chunk_fn, cm):
    tasks = []  # (type, i, j, b0, nb, dur)
    deps = []
    early = []  # per task: list of deps satisfied at producer's early point
    diagx = [-1] * nc
    trsm = {}
    last_upd = {}

    def add(tp, i, j, b0, nb, dur):
        tasks.append((tp, i, j, b0, nb, dur))
        deps.append([])
        early.append([])
        return len(tasks) - 1

    def dep(t, on, is_early=False):
        if on is None or on < 0:
            return
        (early if is_early else deps)[t].append(on)

    def prodL(i, b):
        if i < nc and b == i:
            return diagx[i], False
        if i < nc and b == i - 1:
            return diagx[i], True
        return trsm[(i, b)], False

    by_last = [[] for _ in range(nc)]
    for j in range(1, nc):
        for i in range(j, nr):
            for b0, nb in chunk_fn(i, j):
                by_last[b0 + nb - 1].append((i, j, b0, nb))

    def make_diagx(k):
        t = add(DIAGX, k, k, 0, 0, cm["diag0"] if k == 0 else cm["diagx"])
        diagx[k] = t
        if k >= 1:
            dep(t, diagx[k - 1])
            dep(t, last_upd.get((k, k - 1)))
            dep(t, last_upd.get((k, k)))

    make_diagx(0)
    for k in range(nc):
        for i in range(k + 1, nr):
            if i == k + 1 and i < nc:
                continue
            t = add(TRSM, i, k, 0, 0, cm["trsm"])
            trsm[(i, k)] = t
            dep(t, diagx[k])
            dep(t, last_upd.get((i, k)))
        if k + 1 < nc:
            make_diagx(k + 1)
        for (i, j, b0, nb) in by_last[k]:
            dur = cm["ovh"] + nb * cm["k128"] * (cm["diagf"] if i == j else 1.0)
            if nb == 1:
                dur = cm["ovh1"] + cm["k128"] * (cm["diagf"] if i == j else 1.0)
            t = add(UPD, i, j, b0, nb, dur)
            dep(t, last_upd.get((i, j)))
            for x in (i, j):
                p, e = prodL(x, k)
                dep(t, p, e)
            last_upd[(i, j)] = t
    return tasks, deps, early


def simulate(tasks, deps, early, P, cm):
    n = len(tasks)
    succ = [[] for _ in range(n)]
    esucc = [[] for _ in range(n)]
    indeg = [0] * n
    for t in range(n):
        ds = set(deps[t])
        es = set(early[t]) - ds
        for d in ds:
            succ[d].append(t)
        for d in es:
            esucc[d].append(t)
        indeg[t] = len(ds) + len(es)
    bl = [0.0] * n
    for t in range(n - 1, -1, -1):
        m = 0.0
        for s in succ[t]:
            m = max(m, bl[s])
        for s in esucc[t]:
            m = max(m, bl[s] - (tasks[t][5] - cm["early"]))
        bl[t] = tasks[t][5] + m
    ready = [(-bl[t], t) for t in range(n) if indeg[t] == 0]
    heapq.heapify(ready)
    ev = []  # (time, kind, task) kind 0 = early release, 1 = finish
    free = P
    now = 0.0
    started = 0
    busy = 0.0
    order = []
    while started < n or ev:
        while free > 0 and ready:
            _, t = heapq.heappop(ready)
            order.append(t)
            free -= 1
            started += 1
            d = tasks[t][5]
            busy += d
            heapq.heappush(ev, (now + d, 1, t))
            if esucc[t]:
                heapq.heappush(ev, (now + cm["early"], 0, t))
        if not ev:
            raise RuntimeError("cycle")
        now, kind, t = heapq.heappop(ev)
        lst = succ[t] if kind == 1 else esucc[t]
        if kind == 1:
            free += 1
        for s in lst:
            indeg[s] -= 1
            if indeg[s] == 0:
                heapq.heappush(ready, (-bl[s], s))
    return now, busy / (P * now), bl[0], order


COST = dict(k128=17.1, ovh=6.5, ovh1=5.9, trsm=20.4, diagx=106.0, diag0=70.0, early=20.0, diagf=0.97)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nc", type=int, default=128)
    ap.add_argument("--P", type=int, default=256)
    ap.add_argument("--rule", default="w8")
    ap.add_argument("--near", type=int, default=0)
    ap.add_argument("--first", type=int, default=0)
    for k, v in COST.items():
        ap.add_argument("--" + k, type=float, default=v)
    a = ap.parse_args()
    cm = {k: getattr(a, k) for k in COST}
    if a.rule.startswith("bin"):
        W = int(a.rule[3:])
        fn = lambda i, j: chunks_bin(i, j, W, a.near, a.first)
    elif a.rule.startswith("w"):
        W = int(a.rule[1:])
        fn = lambda i, j: chunks_w(i, j, W)
    else:
        bounds = eval(a.rule)
        fn = lambda i, j: chunks_bounds(i, j, bounds, a.near)
    tasks, deps, early = build(a.nc, a.nc + 1, fn, cm)
    span, util, crit, _ = simulate(tasks, deps, early, a.P, cm)
    print(f"rule={a.rule} tasks={len(tasks)} makespan={span/1e3:.2f} ms util={util:.3f} critical={crit/1e3:.2f} ms")


if __name__ == "__main__":
    main()
