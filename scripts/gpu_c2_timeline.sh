#!/bin/bash
# C2 ms per fit, this tree's library against tools/ab/*.so (alternated), then a kernel +
# memory-copy trace of this tree's fits
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
shopt -s nullglob
O=gpurun_out/${1:-c2tl}
mkdir -p $O
for rep in 1 2 3; do
  for f in tools/ab/*.so; do
    echo -n "$(basename $f) " >> $O/ab.txt
    GPRX_LIB_OVERRIDE=$PWD/$f timeout -k 10 120 python -u scripts/c2_timeline.py 300 1 >> $O/ab.txt 2>&1 || exit 1
  done
  echo -n "tree " >> $O/ab.txt
  timeout -k 10 120 python -u scripts/c2_timeline.py 300 1 >> $O/ab.txt 2>&1 || exit 1
done
cat $O/ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/prof -o c2 -- python3 scripts/c2_timeline.py 30 0 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
find $O/prof -name '*.csv'
