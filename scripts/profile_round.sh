#!/bin/bash
# Round profile on the GPU box: kernel-trace/stats of the default bench command, then two
# separate PMC passes (FETCH_SIZE, WRITE_SIZE) of a short bench run.  Output under
# gpurun_out/; summaries are copied into profiles/ by scripts/prof_summary.py and
# scripts/pmc_traffic.py.  (--build-iters 0: the build-alone timing launches the same kernel
# with BUILD tasks only and would mix short launches into the fit's per-launch statistics.)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o bench -- python3 $R/bench.py --cpu-n 0 --lml 0 --build-iters 0 > $R/gpurun_out/prof_${TAG}.log 2>&1
echo trace=$?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcf_$TAG -o f -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-n 0 --predict-q 1024 --lml 0 --build-iters 0 > $R/gpurun_out/pmcf_${TAG}.log 2>&1
echo fetch=$?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcw_$TAG -o w -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-n 0 --predict-q 1024 --lml 0 --build-iters 0 > $R/gpurun_out/pmcw_${TAG}.log 2>&1
echo write=$?
