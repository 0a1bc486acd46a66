#!/bin/bash
# chunk-rule A/B at one N: the bare factorisation's device time for GPRX_PT_RATIO = 0, 8, 4, 2
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-ratio}
n=${2:-16384}
mkdir -p $O
for r in 0 8 4 2; do
  GPRX_PT_RATIO=$r timeout -k 10 120 python scripts/pt_trace.py $n > $O/r$r.json 2>&1 || exit 1
done
python - "$O" <<'PY'
import json, sys
for r in (0, 8, 4, 2):
    d = json.load(open(f"{sys.argv[1]}/r{r}.json"))
    print(r, round(d["ms_devbench"], 3), d["chain_period_us"], d["busy_per_ms"][-3:], d["chip_ms_idle"], d["chip_ms_wait"])
PY
