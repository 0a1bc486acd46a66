"""Per-type task statistics of sharded-fit timelines (GPRX_DIST_TRACE_FILE dumps, one file per
rank) next to the single-GPU timeline (scripts/pt_trace.py PT_TRACE_OUT npz)."""
import sys
import numpy as np

NAMES = {0: "DIAGX", 1: "TRSM", 2: "UPD", 3: "BUILD"}


def load_rank(path):
    raw = open(path, "rb").read()
    nt, r, g, nc = np.frombuffer(raw[:16], np.int32)
    tasks = np.frombuffer(raw[16:16 + 16 * nt], np.int32).reshape(nt, 4)
    times = np.frombuffer(raw[16 + 16 * nt:16 + 16 * nt + 32 * nt], np.int64).reshape(nt, 4)
    return tasks, times, int(r), int(g), int(nc)


def stats(label, tasks, times, t0=None):
    t0 = times[:, 0].min() if t0 is None else t0
    tk = (times[:, :3] - t0) / 100.0
    typ = tasks[:, 0] & 0xff
    nb = tasks[:, 0] >> 8
    ex = tk[:, 2] - tk[:, 1]
    wt = tk[:, 1] - tk[:, 0]
    P = len(np.unique(times[:, 3] & 0xffff))
    span = tk[:, 2].max()
    out = [f"{label}: span {span:.0f} us, tasks {len(tasks)}, workers {P}, busy {ex.sum() / (span * P):.3f}, "
           f"wait {wt.sum() / (span * P):.3f}"]
    for t in (3, 0, 1, 2):
        sel = typ == t
        if not sel.any():
            continue
        line = f"  {NAMES[t]:5s} n {sel.sum():6d} exec {ex[sel].mean():7.2f} us  wait {wt[sel].mean():7.1f} us  chip {ex[sel].sum() / P / 1e3:6.2f} ms"
        if t == 2:
            per = ex[sel].sum() / nb[sel].sum()
            line += f"  per-panel {per:.2f} us  panels {nb[sel].sum()}"
        out.append(line)
    return "\n".join(out)


if __name__ == "__main__":
    for arg in sys.argv[1:]:
        if arg.endswith(".npz"):
            d = np.load(arg)
            print(stats(arg, d["tasks"], d["times"]))
        else:
            import glob
            files = sorted(glob.glob(arg + ".r*"))
            loaded = [load_rank(f) for f in files]
            t0 = min(x[1][:, 0].min() for x in loaded)
            for (tasks, times, r, g, nc), f in zip(loaded, files):
                print(stats(f"{arg} rank {r}/{g}", tasks, times, t0))
