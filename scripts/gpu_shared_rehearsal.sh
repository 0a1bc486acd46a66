#!/bin/bash
# the N > 1 bench path rehearsed on one GPU: 2 processes (gloo + peer context, IPC mailboxes,
# every rank on device 0 with its share of the CUs), the driver's default arguments
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-shared}
mkdir -p $O
GPRX_DIST_SHARED_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 100)) bench.py --gpus 2 > $O/bench.json 2> $O/bench.err
r=$?
echo rc=$r
grep -v 'amdgpu.ids\|socket.cpp' $O/bench.err | tail -5
python - "$O" <<'PY'
import json, sys
# gloo's connection message can share stdout with the JSON line
d = json.loads([l for l in open(sys.argv[1] + "/bench.json") if l.startswith('{"metric"')][-1])
print(round(d["value"], 2), d["ms_per_step"], d["dist_error"], d["config"]["parallelism"][:40], (d.get("replicas") or {}).get("value"))
for k, v in (d.get("configs") or {}).items():
    print(k, (v or {}).get("value"), (v or {}).get("error"), (v or {}).get("scaling"))
PY
exit $r
