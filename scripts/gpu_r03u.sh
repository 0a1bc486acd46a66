#!/bin/bash
# f32 tile trace at C4's N (the diagonal chain of the f32 path) and the C3 LML phases
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03u
mkdir -p $O
PT_TRACE_DTYPE=0 timeout -k 10 180 python scripts/pt_trace.py 32768 > $O/pt32768_f32.json 2>&1 || exit 1
PT_TRACE_DTYPE=0 timeout -k 10 120 python scripts/pt_trace.py 4096 > $O/pt4096_f32.json 2>&1 || exit 1
timeout -k 10 180 python scripts/lml_time.py > $O/lml.json 2>&1 || exit 1
python - <<'PY'
import json
for f in ("pt32768_f32", "pt4096_f32"):
    d = json.load(open(f"gpurun_out/r03u/{f}.json"))
    print(f, d["ms_devbench"], d["chain_period_us"], d["DIAGX"], d["diagx_phase_us"], d["busy_per_ms"][-6:])
print(open("gpurun_out/r03u/lml.json").read())
PY
