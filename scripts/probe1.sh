set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 200 python scripts/devbench.py all > gpurun_out/devbench_all.json 2>&1
for s in 1 2 4 6; do
  GPRX_DEBUG_SKIP=$s timeout -k 10 100 python scripts/devbench.py potrf > gpurun_out/devbench_skip$s.json 2>&1
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace1 -o t -- python3 $R/bench.py --cpu-n 0 --steps 3 --predict-q 1024 > $R/gpurun_out/trace1.log 2>&1
