#!/bin/bash
# Round-3 profile on the GPU box (gpurun_out/, summaries copied to profiles/ afterwards):
#  1. kernel-trace --stats of the bench headline (the roofline's avg launch is checked against it)
#  2-5. PMC passes, one run each (never combined with traces): FETCH_SIZE, WRITE_SIZE, and the
#     MFMA-busy set, over two C3 fits with the fused build, and FETCH/WRITE over two fits with the
#     covariance build as its own kernel (GPRX_KBUILD=separate: the build-alone launch)
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03b}
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o bench -- python3 $R/bench.py --configs 0 --cpu-n 0 --lml 0 --build-iters 0 --variance-q 0 > $R/gpurun_out/prof_${TAG}.json 2> $R/gpurun_out/prof_${TAG}.err || exit 1
echo trace ok
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcf_$TAG -o f -- python3 $R/scripts/prof_fit.py 16384 > $R/gpurun_out/pmcf_${TAG}.log 2>&1 || exit 1
echo fetch ok
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcw_$TAG -o w -- python3 $R/scripts/prof_fit.py 16384 > $R/gpurun_out/pmcw_${TAG}.log 2>&1 || exit 1
echo write ok
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcm_$TAG -o m -- python3 $R/scripts/prof_fit.py 16384 > $R/gpurun_out/pmcm_${TAG}.log 2>&1 || exit 1
echo mfma ok
GPRX_KBUILD=separate timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcfb_$TAG -o f -- python3 $R/scripts/prof_fit.py 16384 > $R/gpurun_out/pmcfb_${TAG}.log 2>&1 || exit 1
echo fetch-build ok
GPRX_KBUILD=separate timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcwb_$TAG -o w -- python3 $R/scripts/prof_fit.py 16384 > $R/gpurun_out/pmcwb_${TAG}.log 2>&1 || exit 1
echo write-build ok
