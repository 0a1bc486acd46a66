#!/bin/bash
# final evidence of the round: full GPU suite, the default bench line, the kernel-trace stats
# of the bench headline, the back-substitution trace
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${1:-r03ap}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
R=$?
tail -3 $O/gputest.log
[ $R -eq 0 ] || exit $R
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 200 python -u scripts/bs_trace.py > $O/bs_trace_c3.json 2>&1 || exit 1
R0=$PWD
cd /tmp || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R0/$O/prof -o bench -- python3 $R0/bench.py --configs 0 --cpu-n 0 --lml 0 --build-iters 0 --variance-q 0 > $R0/$O/prof_bench.json 2> $R0/$O/prof_bench.err || exit 1
cd $R0
python - "$O" <<'PY'
import json, sys
d = json.load(open(sys.argv[1] + "/bench.json"))
print({k: d[k] for k in ("value", "ms_per_step")}, d["roofline"]["frac"], d["roofline"]["avg_launch_us"], d.get("cpu_baseline", {}).get("value"))
for k, v in (d.get("configs") or {}).items():
    print(k, {x: v.get(x) for x in ("value", "ms_per_step", "error")}, (v.get("roofline") or {}).get("frac"))
print("lml", d.get("lml_grad", {}).get("ms_wall"), "predict", d.get("predict", {}).get("pts_per_s_device"), "phases", d.get("phases"))
PY
find $O/prof -name '*stats*'
