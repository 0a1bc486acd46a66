"""Analyse per-rank device task traces of the distributed fit (GPRX_DIST_TRACE_DEV=<dir>):
per rank, the task timeline {ticket taken, inputs ready, done, workgroup}, long waits and
the DIAGX chain.  Usage: python scripts/dist_trace.py <dir>"""
import glob
import os
import sys

import numpy as np

NAMES = {0: "DIAGX", 1: "TRSM", 2: "UPD", 3: "BUILD"}


def load(path):
    with open(path, "rb") as f:
        ntasks, nc, g, gb = np.frombuffer(f.read(16), np.int32)
        lst = np.frombuffer(f.read(16 * ntasks), np.int32).reshape(ntasks, 4)
        tr = np.frombuffer(f.read(), np.int64).reshape(-1, 4)
    return int(ntasks), int(nc), int(g), int(gb), lst, tr


def main(d):
    ranks = sorted(glob.glob(os.path.join(d, "rank*.bin")))
    data = [load(p) for p in ranks]
    t0 = min(int(tr[:nt, 0][tr[:nt, 0] > 0].min()) for nt, _, _, _, _, tr in data)
    for r, (nt, nc, g, gb, lst, tr) in enumerate(data):
        T = (tr[:nt, :3] - t0) / 100.0  # 100 MHz ticks -> us
        wg = tr[:nt, 3] & 0xFFFF
        typ = lst[:, 0] & 255
        wait = T[:, 1] - T[:, 0]
        exe = T[:, 2] - T[:, 1]
        end = T[:, 2].max()
        print(f"rank {r}: g {g} gb {gb} tasks {nt} span {end:.0f} us, busy {exe.sum() / (end * (wg.max() + 1)):.2f}")
        for ty in range(4):
            m = typ == ty
            if m.any():
                print(f"  {NAMES[ty]:5s} n {m.sum():5d} exec mean {exe[m].mean():8.1f} wait mean {wait[m].mean():8.1f} "
                      f"max {wait[m].max():8.1f}")
        # the longest waits
        idx = np.argsort(-wait)[:8]
        for q in idx:
            t = lst[q]
            print(f"    t{q:5d} {NAMES[t[0] & 255]:5s}({t[1]},{t[2]},b0 {t[3]},nb {t[0] >> 8}) taken {T[q, 0]:9.1f} "
                  f"ready {T[q, 1]:9.1f} done {T[q, 2]:9.1f} wg {wg[q]}")
        # DIAGX chain on this rank
        dm = np.where(typ == 0)[0]
        ks = lst[dm, 1]
        o = np.argsort(ks)
        print("    DIAGX k:ready/done " + " ".join(f"{ks[o][x]}:{T[dm[o][x], 1]:.0f}/{T[dm[o][x], 2]:.0f}"
                                                for x in range(min(12, len(o)))))


if __name__ == "__main__":
    main(sys.argv[1])
