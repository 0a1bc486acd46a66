#!/bin/bash
# The N > 1 bench path rehearsed on ONE GPU with more ranks (GPRX_DIST_SHARED_GPU: every rank on
# device 0, each on 1/world of the CUs, peer context over the socket group).  Usage (from the repo
# root, through gpurun): bash scripts/rehearse.sh TAG WORLD [WORLD ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
TAG=${1:?tag}
shift
O=$PWD/gpurun_out/$TAG
mkdir -p "$O"
for W in "$@"; do
    GPRX_DIST_SHARED_GPU=1 GPU_MAX_HW_QUEUES=${HWQ:-4} timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$W" \
        --master-addr 127.0.0.1 --master-port $((29700 + RANDOM % 200)) bench.py --gpus "$W" --steps 5 --warmup 2 \
        --cpu-n 0 --cpu-lml-ns "" --cpu-predict-q 0 --build-iters 0 > "$O/shared_w$W.json" 2> "$O/shared_w$W.err" \
        || { echo "world $W failed"; tail -n 40 "$O/shared_w$W.err"; exit 1; }
    python scripts/bench_brief.py "$O/shared_w$W.json"
done
echo "rehearsals done"
