#!/bin/bash
# tile traces at N = 4096 / 16384, split diagonal step on and off (GPRX_PT_SPLIT)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-ab}
mkdir -p $O
for n in 4096 16384; do
  timeout -k 10 120 python scripts/pt_trace.py $n > $O/pt$n.json 2>&1 || exit 1
  GPRX_PT_SPLIT=0 timeout -k 10 120 python scripts/pt_trace.py $n > $O/pt${n}_nosplit.json 2>&1 || exit 1
done
python - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for f in ("pt4096", "pt4096_nosplit", "pt16384", "pt16384_nosplit"):
    d = json.load(open(f"{O}/{f}.json"))
    print(f, round(d["ms_devbench"], 3), d.get("chain_period_us"), "DIAGX", round(d["DIAGX"]["exec_us_mean"], 1),
          "TRSM", round(d["TRSM"]["exec_us_mean"], 1), "UPD64", round(d.get("UPD_nb64", {}).get("exec_us_mean", 0), 1),
          {k: round(v["exec_us_mean"], 1) for k, v in d.items() if k.startswith("TPART_c")})
PY
