#!/bin/bash
# two processes on one GPU: the sharded LML at N = 16384 with the window the selection picks
# (mailbox kept below 2 GiB), the sharded-fit GPU tests, the N = 2 bench rehearsal with the LML leg
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r03aq}
mkdir -p $O
port=$((29700 + RANDOM % 200))
GPRX_DIST_VERBOSE=1 timeout -k 5 90 python -u scripts/peer_lml_dbg.py 0 2 $port 16384 40 > $O/r0.txt 2>&1 &
p0=$!
GPRX_DIST_VERBOSE=1 timeout -k 5 90 python -u scripts/peer_lml_dbg.py 1 2 $port 16384 40 > $O/r1.txt 2>&1 &
p1=$!
wait $p0; r0=$?; wait $p1; r1=$?
echo "peer lml rc $r0 $r1"
grep -v "amdgpu.ids\|socket.cpp\|Gloo" $O/r0.txt | grep -v 'ipc handle opened' | tail -16
[ $r0 -eq 0 ] && [ $r1 -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $O/gputest_dist.log 2>&1 || { tail -20 $O/gputest_dist.log; exit 1; }
tail -2 $O/gputest_dist.log
GPRX_DIST_SHARED_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 100)) bench.py --gpus 2 --dist-lml 1 > $O/bench2.json 2> $O/bench2.err || { tail -5 $O/bench2.err; exit 1; }
python - "$O" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1] + "/bench2.json") if l.startswith('{"metric"')][-1])
print(round(d["value"], 2), d["ms_per_step"], d.get("dist_error"), "sharded lml ms", d.get("lml_grad_sharded_ms_wall"))
for k, v in (d.get("configs") or {}).items():
    print(k, (v or {}).get("value"), (v or {}).get("error"), (v or {}).get("dist"))
PY
