#!/bin/bash
# tile trace at one N for several library builds (tools/ab/*.so) and this tree's
cd "$GRAFT_REPO_ROOT" || exit 1
shopt -s nullglob
O=gpurun_out/${1:-libs}
n=${2:-16384}
mkdir -p $O
for f in tools/ab/*.so; do
  b=$(basename $f .so)
  GPRX_LIB_OVERRIDE=$PWD/$f timeout -k 10 120 python scripts/pt_trace.py $n > $O/$b.json 2>&1 || exit 1
done
timeout -k 10 120 python scripts/pt_trace.py $n > $O/tree.json 2>&1 || exit 1
GPRX_PT_SPLIT=0 timeout -k 10 120 python scripts/pt_trace.py $n > $O/tree_nosplit.json 2>&1 || exit 1
python - "$O" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.load(open(f))
    print(os.path.basename(f), round(d["ms_devbench"], 3), round(d["clock_ghz_median"], 2), d.get("chain_period_us"), "DIAGX",
          round(d["DIAGX"]["exec_us_mean"], 1), "TRSM", round(d["TRSM"]["exec_us_mean"], 1),
          "UPD1", round(d.get("UPD_nb1", {}).get("exec_us_mean", 0), 1),
          "UPD64", round(d.get("UPD_nb64", {}).get("exec_us_mean", 0), 1),
          {k: round(v["exec_us_mean"], 1) for k, v in d.items() if k.startswith("TPART_c")})
PY
