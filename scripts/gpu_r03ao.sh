#!/bin/bash
# full GPU suite, back-substitution traces, then the C3 bench leg and C2 fits of this tree
# against tools/ab/*.so
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r03ao}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
R=$?
tail -4 $O/gputest.log
[ $R -eq 0 ] || exit $R
timeout -k 10 200 python -u scripts/bs_trace.py > $O/bs_trace_c3.json 2>&1 || exit 1
timeout -k 10 100 python -u scripts/bs_trace.py 4096 > $O/bs_trace_c2.json 2>&1 || exit 1
cat $O/bs_trace_c3.json $O/bs_trace_c2.json
shopt -s nullglob
Q="--cpu-n 0 --lml 0 --variance-q 0 --predict-q 0 --build-iters 0 --configs 0 --steps 20"
for rep in 1 2 3; do
  for f in tools/ab/*.so; do
    echo -n "$(basename $f) " >> $O/c2ab.txt
    GPRX_LIB_OVERRIDE=$PWD/$f timeout -k 10 120 python -u scripts/c2_timeline.py 300 1 >> $O/c2ab.txt 2>&1 || exit 1
    GPRX_LIB_OVERRIDE=$PWD/$f timeout -k 10 300 python bench.py $Q > $O/c3_$(basename $f .so)_$rep.json 2>/dev/null || exit 1
  done
  echo -n "tree " >> $O/c2ab.txt
  timeout -k 10 120 python -u scripts/c2_timeline.py 300 1 >> $O/c2ab.txt 2>&1 || exit 1
  timeout -k 10 300 python bench.py $Q > $O/c3_tree_$rep.json 2>/dev/null || exit 1
done
cat $O/c2ab.txt
python - "$O" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/c3_*.json")):
    d = json.load(open(f))
    print(os.path.basename(f), round(d["value"], 3), d["ms_per_step"], round(d["roofline"]["avg_launch_us"], 1), d["phases"]["backsolve"]["ms_per_fit"])
PY
