#!/bin/bash
# full GPU suite, default bench (C3 headline + C2/C4/C5), sharded timings on virtual ranks
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r03p}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
R=$?
tail -4 $O/gputest.log
[ $R -eq 0 ] || exit $R
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 python -u scripts/dist_time.py 16384 5 single v1 v2 v4 v8 > $O/dist_time.jsonl 2>&1 || exit 1
cut -c1-200 $O/dist_time.jsonl
python - "$O" <<'PY'
import json, sys
d = json.load(open(sys.argv[1] + "/bench.json"))
print({k: d[k] for k in ("value", "ms_per_step")}, d["roofline"]["frac"], d["roofline"]["avg_launch_us"], d.get("cpu_baseline"))
for k, v in (d.get("configs") or {}).items():
    print(k, {x: v.get(x) for x in ("value", "ms_per_step", "error")}, (v.get("roofline") or {}).get("frac"))
PY
