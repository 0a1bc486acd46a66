#!/bin/bash
# the same tile trace with the previous commit's library (tools/ab/libgprx_head.so) and this tree's
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-headab}
mkdir -p $O
for n in 4096 16384; do
  GPRX_LIB_OVERRIDE=$PWD/tools/ab/libgprx_head.so timeout -k 10 120 python scripts/pt_trace.py $n > $O/pt${n}_head.json 2>&1 || exit 1
  GPRX_PT_SPLIT=0 timeout -k 10 120 python scripts/pt_trace.py $n > $O/pt${n}_nosplit.json 2>&1 || exit 1
  timeout -k 10 120 python scripts/pt_trace.py $n > $O/pt${n}.json 2>&1 || exit 1
done
python - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for n in (4096, 16384):
    for f in (f"pt{n}_head", f"pt{n}_nosplit", f"pt{n}"):
        d = json.load(open(f"{O}/{f}.json"))
        print(f, round(d["ms_devbench"], 3), round(d["clock_ghz_median"], 2), d.get("chain_period_us"), "DIAGX",
              round(d["DIAGX"]["exec_us_mean"], 1), "TRSM", round(d["TRSM"]["exec_us_mean"], 1),
              "UPD64", round(d.get("UPD_nb64", {}).get("exec_us_mean", 0), 1),
              {k: round(v["exec_us_mean"], 1) for k, v in d.items() if k.startswith("TPART_c")})
PY
