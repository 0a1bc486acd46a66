#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/dist_f32_determinism.py > gpurun_out/f32det.jsonl 2>&1; R=$?
python -c "
import json
for l in open('gpurun_out/f32det.jsonl'):
    if l.startswith('{'):
        d = json.loads(l); print(d['g'], d['steps'], d['distinct'], sorted(set(tuple(r[1:]) for r in d['runs'])))
"
[ $R -eq 0 ] || exit $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -q --timeout 200 --timeout-method thread > gpurun_out/dbg_dist.log 2>&1; R=$?
grep -n "^E  \|passed\|failed\|gprx dist timeout" gpurun_out/dbg_dist.log | cut -c1-300 | tail -20; exit $R
