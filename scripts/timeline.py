#!/usr/bin/env python3
"""Critical-path view of one fit from a rocprofv3 kernel trace (bench_kernel_trace.csv):
per outer panel, the time spent in the panel chain (diag/trsm/inner on the main stream)
and what the look-ahead stream ran meanwhile."""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows = [r for r in rows if r["Kind"] == "KERNEL_DISPATCH"]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # pick the last complete fit: the last kbuild ... last backsolve_alpha
    kb = [i for i, r in enumerate(rows) if "kbuild_kernel" in r["Kernel_Name"]]
    start = kb[-2] if len(kb) > 1 else kb[-1]
    fit = []
    for r in rows[start:]:
        fit.append(r)
        if "fit_reduce" in r["Kernel_Name"]:
            break
    t0 = int(fit[0]["Start_Timestamp"])
    by_q = defaultdict(float)
    names = defaultdict(lambda: [0, 0.0])
    for r in fit:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        q = r["Queue_Id"]
        by_q[q] += d
        nm = r["Kernel_Name"].split("(")[0].replace("void gprx::", "")
        key = (nm, r["Grid_Size_X"] if "gemm" in nm else "")
        names[nm][0] += 1
        names[nm][1] += d
    t1 = max(int(r["End_Timestamp"]) for r in fit)
    print(f"fit span {(t1 - t0) / 1e3:.1f} us, kernels {len(fit)}")
    for q, v in sorted(by_q.items()):
        print(f"  queue {q}: busy {v:.1f} us")
    for k, (c, v) in sorted(names.items(), key=lambda x: -x[1][1]):
        print(f"  {k:60s} n={c:4d} sum={v:9.1f} us avg={v / c:8.1f}")
    # diag-to-diag gaps on the main queue
    diag = [r for r in fit if "diag_potrf" in r["Kernel_Name"]]
    gaps = []
    for a, b in zip(diag, diag[1:]):
        gaps.append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in diag]
    print(f"diag: n={len(diag)} mean dur {sum(durs) / len(durs):.1f} us, mean gap to next diag {sum(gaps) / len(gaps):.1f} us")
    print("per outer panel (4 diags): span from first diag start to next panel's first diag start")
    for k in range(0, len(diag) - 4, 16):
        a, b = diag[k], diag[k + 4]
        print(f"  panel {k // 4:3d}: {(int(b['Start_Timestamp']) - int(a['Start_Timestamp'])) / 1e3:8.1f} us"
              f"  diag durs {[round(x) for x in durs[k:k + 4]]}  gaps {[round(x) for x in gaps[k:k + 4]]}")


if __name__ == "__main__":
    main()
