#!/bin/bash
# Fit time under tile-schedule parameter variants (env knobs of k_ptiles.hip Params).
# Output: gpurun_out/sweep.log, one "<variant> <fits/s> <potrf avg us>" line per run.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
out=$R/gpurun_out/sweep.log
: > $out
VARS=("base" "GPRX_PT_DIAGX_US=96" "GPRX_PT_W=64" "GPRX_PT_NEAR=2" "GPRX_PT_NEAR=0" "GPRX_PT_W=16")
[ -n "$SWEEP" ] && read -r -a VARS <<< "$SWEEP"
for v in "${VARS[@]}"; do
  if [ "$v" = base ]; then envs=""; else envs="${v//,/ }"; fi  # a,b: several knobs
  line=$(env $envs timeout -k 10 120 python -u $R/bench.py --cpu-n 0 --lml 0 --predict-q 1024 --steps 20 2>/dev/null | tail -1) || exit 1
  echo "$v $(echo "$line" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["value"],3), round(d["roofline"]["avg_launch_us"],1))')" >> $out
done
cat $out
