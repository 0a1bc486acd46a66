#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE: separate
runs, MI355X_MICROARCH.md "rocprofv3 PMC slots").  The figures are L2-fabric bytes (the L2's
memory-side requests: Infinity-Cache hits are counted, so they bound HBM from above).
FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads on gfx950 (guide §HBM):
the tile kernels' operand feed is exactly that (`global_load_lds` 16 B per lane, all of
their bulk reads), so "fetch_bytes_per_launch_corrected" doubles it; the raw counter is
kept beside it ("fetch_bytes_per_launch_raw") for kernels whose reads are narrower.
Both counters are in KB (rocprofv3 derived metrics).  Writes profiles/<tag>_pmc_traffic.json.

    python scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/r01_pmc_traffic.json
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.match(r"(?:void )?(?:[A-Za-z_0-9]+::)*([A-Za-z_0-9]+<[^()]*>|[A-Za-z_0-9]+)", name)
    return m.group(1) if m else name


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    acc = defaultdict(lambda: [0.0, 0])
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") != counter:
                    continue
                k = short(r["Kernel_Name"])
                acc[k][0] += float(r["Counter_Value"])
                acc[k][1] += 1
    return acc


def main():
    fdir, wdir, out = sys.argv[1:4]
    fe, wr = load(fdir, "FETCH_SIZE"), load(wdir, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fe) | set(wr)):
        f, nf = fe.get(k, [0.0, 0])
        w, nw = wr.get(k, [0.0, 0])
        n = max(nf, nw, 1)
        fb = 2.0 * f * 1024 / max(nf, 1)
        wb = w * 1024 / max(nw, 1)
        res[k] = {"launches": n, "fetch_bytes_per_launch_raw": fb / 2, "fetch_bytes_per_launch_corrected": fb,
                  "write_bytes_per_launch": wb, "hbm_bytes_per_launch": fb + wb}
    json.dump({"counters": "L2-fabric bytes (MALL hits included): FETCH_SIZE x 2 (gfx950, 16 B/lane streaming "
               "reads) + WRITE_SIZE, KB -> bytes; raw FETCH_SIZE kept", "kernels": res},
              open(out, "w"), indent=1)
    print(json.dumps(res, indent=1)[:3000])


if __name__ == "__main__":
    main()
