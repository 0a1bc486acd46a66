#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for N in 4096 8192 16384; do
  PT_TRACE_OUT=gpurun_out/pt$N.npz timeout -k 10 120 python -u scripts/pt_trace.py $N > gpurun_out/pt$N.json 2>&1 || exit 1
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/pt$N.json').read()[open('gpurun_out/pt$N.json').read().index('{'):])
print($N, 'span', d['span_us'], 'devbench_ms', d['ms_devbench'], 'diagx', d['diagx_exec_mean_us'], 'gap', d['diagx_gap_mean_us'], 'tasks', d['tasks'])"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -x --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1; R=$?
tail -2 gpurun_out/par.log; exit $R
