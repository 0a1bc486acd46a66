#!/usr/bin/env python3
"""Per-kernel summary of any rocprofv3 PMC pass(es): every counter averaged over the launches of
each kernel, with the launch duration and the clock (GRBM_GUI_ACTIVE is summed over the 8 XCDs,
so clock = GRBM_GUI_ACTIVE / 8 / duration; MI355X_MICROARCH.md, DVFS give-back).  SQ_WAVE_CYCLES,
SQ_WAIT_*, SQ_ACTIVE_INST_* and SQ_BUSY_CYCLES count quad-cycles (the guide's cycle-constants
table); SQ_VALU_MFMA_BUSY_CYCLES counts cycles.  Derived fractions per kernel:
  mfma_busy_frac   = MFMA_BUSY / (clock cycles x 1024 SIMDs)
  valu_active_frac = 4 ACTIVE_INST_VALU / (clock cycles x 1024)   (issue cycles of VALU instructions)
  wait_inst_frac   = WAIT_INST_ANY / WAVE_CYCLES, wait_any_frac = WAIT_ANY / WAVE_CYCLES,
  active_any_frac  = ACTIVE_INST_ANY / WAVE_CYCLES (the three are disjoint: guide's PMC table)
  lds_conflict_frac = LDS_BANK_CONFLICT / LDS_IDX_ACTIVE

    python scripts/pmc_generic.py OUT.json DIR [DIR ...] [--kernel SUBSTR]
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
    args = sys.argv[1:]
    filt = None
    if "--kernel" in args:
        i = args.index("--kernel")
        filt = args[i + 1]
        del args[i:i + 2]
    out, dirs = args[0], args[1:]
    per = defaultdict(lambda: defaultdict(dict))  # kernel -> (dir, dispatch) -> counters
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                if filt and filt not in k:
                    continue
                c = per[k][(d, int(r["Dispatch_Id"]))]
                c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                c["dur_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
                c["grbm_" + d] = c.get("GRBM_GUI_ACTIVE", 0.0)
    res = {}
    for k, launches in per.items():
        names = sorted({n for c in launches.values() for n in c if n.isupper() or n.startswith("SQ_")})
        avg = {n: float(sum(c.get(n, 0.0) for c in launches.values() if n in c)
                        / max(1, sum(1 for c in launches.values() if n in c))) for n in names}
        dur = float(sum(c["dur_ns"] for c in launches.values()) / len(launches))
        ent = {"launches": len(launches), "dur_ms_mean": dur * 1e-6, "counters_mean": avg}
        g = avg.get("GRBM_GUI_ACTIVE")
        if g:
            cyc = g / 8.0
            ent["clock_ghz"] = cyc / dur
            simd_cyc = cyc * 1024
            if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
                ent["mfma_busy_frac"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cyc
            if "SQ_ACTIVE_INST_VALU" in avg:
                ent["valu_active_frac"] = 4.0 * avg["SQ_ACTIVE_INST_VALU"] / simd_cyc
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            for n, key in (("SQ_WAIT_INST_ANY", "wait_inst_frac"), ("SQ_WAIT_ANY", "wait_any_frac"),
                           ("SQ_ACTIVE_INST_ANY", "active_any_frac"), ("SQ_ACTIVE_INST_VALU", "active_valu_of_wave"),
                           ("SQ_WAIT_INST_LDS", "wait_inst_lds_frac")):
                if n in avg:
                    ent[key] = avg[n] / wc
        if avg.get("SQ_LDS_IDX_ACTIVE"):
            ent["lds_conflict_frac"] = avg.get("SQ_LDS_BANK_CONFLICT", 0.0) / avg["SQ_LDS_IDX_ACTIVE"]
        res[k] = ent
    json.dump({"sources": [os.path.basename(d.rstrip("/")) for d in dirs], "kernels": res}, open(out, "w"), indent=1)
    for k, v in res.items():
        print(k, json.dumps({x: y for x, y in v.items() if x != "counters_mean"}))


if __name__ == "__main__":
    main()
