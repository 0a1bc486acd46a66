"""Summarise a rocprofv3 run (rocpd SQLite output, or a *_kernel_stats.csv) into the
per-kernel stats table committed under profiles/.

    python scripts/prof_summary.py gpurun_out/prof6/run_results.db > profiles/r01_bench_kernel_stats.csv
"""
import csv
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    return [(n, int(k), float(t), float(a), float(p)) for n, k, t, a, p in rows]


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3,
                        float(r["Percentage"])))
    return out


def main():
    src = sys.argv[1]
    rows = from_db(src) if src.endswith(".db") else from_csv(src)
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "calls", "total_us", "avg_us", "percent"])
    for n, k, t, a, p in rows:
        w.writerow([n, k, f"{t:.3f}", f"{a:.3f}", f"{p:.2f}"])


if __name__ == "__main__":
    main()
