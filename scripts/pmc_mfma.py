#!/usr/bin/env python3
"""MFMA-busy summary of a rocprofv3 PMC pass (SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES,
SQ_WAVE_CYCLES, GRBM_GUI_ACTIVE), per kernel and launch.  GRBM_GUI_ACTIVE is summed over the
8 XCDs (MI355X_MICROARCH.md, DVFS give-back), so clock = GRBM_GUI_ACTIVE / 8 / duration.
mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 256 CUs * 4 SIMDs): the
fraction of SIMD-cycles of the launch with the matrix pipe busy (the counter counts cycles,
the guide's calibration table).
    python scripts/pmc_mfma.py gpurun_out/pmcm_r03b profiles/r03b_pmc_mfma.json
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


def main():
    d, out = sys.argv[1:3]
    rows = defaultdict(dict)  # (kernel, dispatch) -> counters
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            key = (short(r["Kernel_Name"]), int(r["Dispatch_Id"]))
            rows[key][r["Counter_Name"]] = float(r["Counter_Value"])
            rows[key]["dur_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    res = defaultdict(list)
    for (k, disp), c in sorted(rows.items(), key=lambda x: x[0][1]):
        g = c.get("GRBM_GUI_ACTIVE", 0.0)
        if not g:
            continue
        cyc = g / 8.0
        res[k].append({
            "dispatch": disp, "dur_ms": c["dur_ns"] * 1e-6, "clock_ghz": cyc / c["dur_ns"],
            "mfma_busy_cycles": c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0),
            "mfma_busy_frac": c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (cyc * 256 * 4),
            "sq_busy_frac": c.get("SQ_BUSY_CYCLES", 0.0) / (cyc * 32),
            "wave_cycles": c.get("SQ_WAVE_CYCLES", 0.0)})
    json.dump({"counters": "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE",
               "normalisation": "mfma_busy_frac = MFMA_BUSY / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs); "
                                "sq_busy_frac = SQ_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 32 SEs: 8 XCDs x 4)",
               "kernels": res}, open(out, "w"), indent=1)
    for k, v in res.items():
        if "potrf" in k or "kbuild" in k or "mfma" in k:
            for x in v:
                print(k, json.dumps(x))


if __name__ == "__main__":
    main()
