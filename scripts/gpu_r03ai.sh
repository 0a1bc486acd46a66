#!/bin/bash
# f32 split step: traces at 4096 / 32768 (split on / off), then the factorisation GPU tests
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r03ai}
mkdir -p $O
for n in 4096 32768; do
  PT_TRACE_DTYPE=0 timeout -k 10 150 python scripts/pt_trace.py $n > $O/f32_$n.json 2>&1 || { tail -5 $O/f32_$n.json; exit 1; }
  PT_TRACE_DTYPE=0 GPRX_PT_SPLIT=0 timeout -k 10 150 python scripts/pt_trace.py $n > $O/f32_${n}_nosplit.json 2>&1 || exit 1
done
python - "$O" <<'PY'
import json, sys
for f in ("f32_4096", "f32_4096_nosplit", "f32_32768", "f32_32768_nosplit"):
    d = json.load(open(f"{sys.argv[1]}/{f}.json"))
    print(f, round(d["ms_devbench"], 3), d["chain_period_us"], round(d["DIAGX"]["exec_us_mean"], 1), d.get("split_step_us", {}).get("diagx"))
PY
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiles.py tests/test_gpu_configs.py tests/test_gpu_dist.py -x -q \
  --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
R=$?
tail -3 $O/gputest.log
exit $R
