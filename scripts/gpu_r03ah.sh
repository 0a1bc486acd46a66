#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r03ah
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -q -k "peer" --timeout 250 --timeout-method thread > gpurun_out/r03ah/t.log 2>&1
R=$?; tail -5 gpurun_out/r03ah/t.log; exit $R
