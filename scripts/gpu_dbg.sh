#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -q -x --timeout 200 --timeout-method thread > gpurun_out/dbg_dist.log 2>&1; R=$?
grep -n "^E  \|passed\|failed\|gprx dist timeout" gpurun_out/dbg_dist.log | cut -c1-300 | tail -8
[ $R -eq 0 ] || exit $R
GPRX_DIST_TRACE_FILE=gpurun_out/dx_v2 timeout -k 10 200 python -u scripts/dist_time.py 16384 3 v2 > /dev/null 2>&1 || exit 1
python3 scripts/dist_trace_stats.py gpurun_out/dx_v2 | grep -E "UPD|rank 0"
timeout -k 10 300 python -u scripts/dist_time.py 16384 5 single v1 v2 v4 v8 > gpurun_out/dt16384.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u scripts/dist_time.py 4096 10 single v1 v2 v4 > gpurun_out/dt4096.jsonl 2>&1 || exit 1
python3 -c "
import json
for f in ('gpurun_out/dt4096.jsonl','gpurun_out/dt16384.jsonl'):
    for l in open(f):
        if l.startswith('{'):
            d=json.loads(l); print(d['n'], d['mode'], round(d['ms_per_fit'],2), round(d['ms_factor_kernel'],2), round(d['ms_solve'],3), d.get('dist',{}).get('est_us'), d['alpha_vs_first'])
"
