#!/bin/bash
# C3 bench leg (no CPU baseline, no extras) with each tools/ab/*.so and this tree's library,
# alternated twice on the same box
cd "$GRAFT_REPO_ROOT" || exit 1
shopt -s nullglob
O=gpurun_out/${1:-benchab}
mkdir -p $O
Q="--cpu-n 0 --lml 0 --variance-q 0 --predict-q 0 --build-iters 0 --configs 0 --steps 20"
for rep in 1 2; do
  for f in tools/ab/*.so; do
    b=$(basename $f .so)
    GPRX_LIB_OVERRIDE=$PWD/$f timeout -k 10 300 python bench.py $Q > $O/${b}_$rep.json 2>/dev/null || exit 1
  done
  timeout -k 10 300 python bench.py $Q > $O/tree_$rep.json 2>/dev/null || exit 1
done
python - "$O" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.load(open(f))
    print(os.path.basename(f), round(d["value"], 2), round(d["roofline"]["avg_launch_us"], 1))
PY
