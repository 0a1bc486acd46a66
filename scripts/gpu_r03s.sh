#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiles.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
R=$?
tail -2 $O/gputest.log
[ $R -eq 0 ] || exit $R
timeout -k 10 600 python -u bench.py --cpu-n 0 --lml 0 --variance-q 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r03s/bench.json"))
print({k: d[k] for k in ("value", "ms_per_step")}, d["roofline"]["frac"], d["roofline"]["avg_launch_us"])
for k, v in (d.get("configs") or {}).items():
    print(k, v.get("value"), v.get("ms_per_step"), (v.get("roofline") or {}).get("avg_launch_us"))
PY
