#!/bin/bash
# sharded-fit timings at C3 (N = 16384) and N = 4096: single vs virtual ranks, LML
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/dist_time.py 16384 5 single rccl1 v1 v2 v4 v8 > gpurun_out/dist_time_16384.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u scripts/dist_time.py 4096 10 single v1 v2 v4 > gpurun_out/dist_time_4096.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u scripts/dist_time.py 16384 3 lml:single lml:v1 lml:v2 lml:v4 > gpurun_out/dist_lml_16384.jsonl 2>&1 || exit 1
cat gpurun_out/dist_time_16384.jsonl gpurun_out/dist_time_4096.jsonl gpurun_out/dist_lml_16384.jsonl | cut -c1-400
