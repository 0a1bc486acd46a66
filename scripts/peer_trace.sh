#!/bin/bash
# WORLD processes on one GPU run scripts/peer_fit_trace.py (N, fits); traces under gpurun_out/TAG.
# Usage: bash scripts/peer_trace.sh TAG WORLD N FITS
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
TAG=${1:?tag}; W=${2:?world}; N=${3:-16384}; F=${4:-3}
O=$PWD/gpurun_out/$TAG
mkdir -p "$O"
PORT=$((29900 + RANDOM % 90))
pids=()
for ((r = 0; r < W; r++)); do
    timeout -k 10 300 python -u scripts/peer_fit_trace.py $r $W $PORT $N $F "$O/trace_w${W}" > "$O/peer_w${W}_r$r.log" 2>&1 &
    pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
cat "$O"/peer_w${W}_r*.log | grep -v amdgpu.ids
exit $rc
