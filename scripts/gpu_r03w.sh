#!/bin/bash
# traces (split on / off) at 4096 and 16384, factorisation tests, then the bench (no CPU leg)
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r03w}
bash scripts/gpu_trace_libs.sh $T 4096 || exit 1
bash scripts/gpu_trace_libs.sh ${T}16 16384 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiles.py tests/test_gpu_configs.py tests/test_gpu_dist.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/$T/gputest.log 2>&1
R=$?
tail -2 gpurun_out/$T/gputest.log
[ $R -eq 0 ] || exit $R
timeout -k 10 600 python -u bench.py --cpu-n 0 --lml 0 --variance-q 0 > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
python - $T <<'PY'
import json, sys
T = sys.argv[1]
d = json.load(open(f"gpurun_out/{T}/bench.json"))
print({k: d[k] for k in ("value", "ms_per_step")}, d["roofline"]["frac"], d["roofline"]["avg_launch_us"])
for k, v in (d.get("configs") or {}).items():
    print(k, v.get("value"), v.get("ms_per_step"), (v.get("roofline") or {}).get("avg_launch_us"))
d = json.load(open(f"gpurun_out/{T}/tree.json"))
print(json.dumps(d.get("split_step_us")))
PY
