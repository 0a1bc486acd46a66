#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
: > gpurun_out/triage.jsonl
export GPRX_DIST_CHECK=1
for args in "16384 2,3,4,5,6,7,8" "16384 8 16" "16384 4 8" "8192 3,5,7 4" "4096 8 2"; do
  timeout -k 10 200 python -u scripts/dist_triage.py $args >> gpurun_out/triage.jsonl 2>&1 || { echo "FAILED $args"; break; }
done
cut -c1-200 gpurun_out/triage.jsonl
