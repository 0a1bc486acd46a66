#!/bin/bash
# full GPU suite, then the default bench (C3 headline + configs), then sharded timings
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r03c.log 2>&1
R=$?
tail -4 gpurun_out/gputest_r03c.log
[ $R -eq 0 ] || exit $R
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r03c.json 2> gpurun_out/bench_r03c.err || { tail -20 gpurun_out/bench_r03c.err; exit 1; }
timeout -k 10 300 python -u scripts/dist_time.py 16384 5 single v1 v2 v4 v8 > gpurun_out/dist_time_r03c.jsonl 2>&1 || exit 1
cut -c1-300 gpurun_out/dist_time_r03c.jsonl
python - <<'PY'
import json
d = json.load(open("gpurun_out/bench_r03c.json"))
print({k: d[k] for k in ("value", "ms_per_step", "roofline")})
for k, v in (d.get("configs") or {}).items():
    print(k, {x: v.get(x) for x in ("value", "ms_per_step", "roofline", "cpu_baseline", "error")})
PY
