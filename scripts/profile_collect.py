#!/usr/bin/env python3
"""Turn the output of `scripts/gpu.sh TAG profile` (merged back under gpurun_out/TAG/) into the
committed summaries that bench.py attaches to its roofline objects:

  profiles/TAG_<leg>_kernel_stats.csv   rocprofv3 --kernel-trace --stats of one bench leg
  profiles/TAG_<leg>_pmc_traffic.json   FETCH_SIZE x 2 + WRITE_SIZE per launch (scripts/pmc_traffic.py)
  profiles/TAG_<leg>_pmc_mfma.json      MFMA-busy fraction per launch (scripts/pmc_mfma.py)

    python scripts/profile_collect.py r04a
"""
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles")
    for d in sorted(glob.glob(os.path.join(src, "prof_*"))):
        if not os.path.isdir(d):
            continue
        leg = os.path.basename(d)[len("prof_"):]
        stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
        if stats:
            shutil.copy(stats[0], os.path.join(dst, f"{tag}_{leg}_kernel_stats.csv"))
            print("stats", leg, stats[0])
    for leg in ("c3", "build"):
        f, w = os.path.join(src, f"pmcf_{leg}"), os.path.join(src, f"pmcw_{leg}")
        if os.path.isdir(f) and os.path.isdir(w):
            subprocess.check_call([sys.executable, os.path.join(ROOT, "scripts", "pmc_traffic.py"), f, w,
                                   os.path.join(dst, f"{tag}_{leg}_pmc_traffic.json")], stdout=subprocess.DEVNULL)
            print("traffic", leg)
    pp = os.path.join(src, "predict_pmc.json")  # (scripts/pmc_generic.py: the predict kernel's issue split)
    if os.path.isfile(pp):
        shutil.copy(pp, os.path.join(dst, f"{tag}_predict_pmc.json"))
        print("pmc predict")
    for leg in ("c3", "c4"):
        m = os.path.join(src, f"pmcm_{leg}")
        if os.path.isdir(m):
            subprocess.check_call([sys.executable, os.path.join(ROOT, "scripts", "pmc_mfma.py"), m,
                                   os.path.join(dst, f"{tag}_{leg}_pmc_mfma.json")], stdout=subprocess.DEVNULL)
            print("mfma", leg)


if __name__ == "__main__":
    main()
