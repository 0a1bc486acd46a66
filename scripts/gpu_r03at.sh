#!/bin/bash
# end of round: full GPU suite, smoke(), and the N = 2 bench path rehearsed on one GPU
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r03at}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
R=$?
tail -2 $O/gputest.log
[ $R -eq 0 ] || exit $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash scripts/gpu_shared_rehearsal.sh ${1:-r03at}_shared
