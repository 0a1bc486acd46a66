#!/bin/bash
# full GPU suite, then C2 ms per fit of this tree against tools/ab/*.so
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r03am}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
R=$?
tail -4 $O/gputest.log
[ $R -eq 0 ] || exit $R
shopt -s nullglob
for rep in 1 2 3; do
  for f in tools/ab/*.so; do
    echo -n "$(basename $f) " >> $O/c2ab.txt
    GPRX_LIB_OVERRIDE=$PWD/$f timeout -k 10 120 python -u scripts/c2_timeline.py 300 1 >> $O/c2ab.txt 2>&1 || exit 1
  done
  echo -n "tree " >> $O/c2ab.txt
  timeout -k 10 120 python -u scripts/c2_timeline.py 300 1 >> $O/c2ab.txt 2>&1 || exit 1
done
cat $O/c2ab.txt
