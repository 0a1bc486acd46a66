#!/bin/bash
# sharded-fit timings (virtual ranks) with each tools/ab/*.so and this tree's library, same box
cd "$GRAFT_REPO_ROOT" || exit 1
shopt -s nullglob
O=gpurun_out/${1:-distab}
mkdir -p $O
for f in tools/ab/*.so; do
  b=$(basename $f .so)
  GPRX_LIB_OVERRIDE=$PWD/$f timeout -k 10 300 python -u scripts/dist_time.py 16384 5 v1 v8 > $O/$b.jsonl 2>&1 || exit 1
done
timeout -k 10 300 python -u scripts/dist_time.py 16384 5 v1 v8 > $O/tree.jsonl 2>&1 || exit 1
for f in $O/*.jsonl; do echo $f; cut -c1-120 $f; done
