#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_trace_libs.sh r03v 4096 || exit 1
bash scripts/gpu_trace_libs.sh r03v16 16384 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiles.py tests/test_gpu_configs.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r03v/gputest.log 2>&1
R=$?
tail -3 gpurun_out/r03v/gputest.log
exit $R
