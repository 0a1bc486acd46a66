#!/bin/bash
# two processes on one GPU: the sharded fit at N = 32768 fp64 (each rank's storage ~2.1 GB, no
# longer mapped by the peer), then the sharded-fit GPU tests
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r03as}
mkdir -p $O
port=$((29700 + RANDOM % 200))
GPRX_DIST_VERBOSE=1 timeout -k 5 100 python -u scripts/peer_lml_dbg.py 0 2 $port 32768 50 fit > $O/r0.txt 2>&1 &
p0=$!
GPRX_DIST_VERBOSE=1 timeout -k 5 100 python -u scripts/peer_lml_dbg.py 1 2 $port 32768 50 fit > $O/r1.txt 2>&1 &
p1=$!
wait $p0; r0=$?; wait $p1; r1=$?
echo "peer fit rc $r0 $r1"
grep -v "amdgpu.ids\|socket.cpp\|Gloo" $O/r0.txt | tail -8
[ $r0 -eq 0 ] && [ $r1 -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $O/gputest_dist.log 2>&1 || { tail -20 $O/gputest_dist.log; exit 1; }
tail -2 $O/gputest_dist.log
