#!/bin/bash
# capped chunk rule only in the last T column blocks: device time at one N
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-tail}
n=${2:-16384}
mkdir -p $O
for cfg in "0 0" "2 16" "2 32" "4 24" "4 48" "8 32"; do
  set -- $cfg
  GPRX_PT_RATIO=$1 GPRX_PT_TAIL=$2 timeout -k 10 120 python scripts/pt_trace.py $n > $O/r$1_t$2.json 2>&1 || exit 1
done
python - "$O" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/r*.json")):
    d = json.load(open(f))
    print(os.path.basename(f), round(d["ms_devbench"], 3), round(d["chain_period_us"]["last16_mean"], 1), d["busy_per_ms"][-3:], d["tasks"])
PY
