#!/bin/bash
# the sharded fit's GPU tests alone (tests/test_gpu_dist.py), verbose, bounded
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 240 --timeout-method thread "$@" > gpurun_out/gpu_dist.log 2>&1
R=$?
tail -40 gpurun_out/gpu_dist.log
exit $R
