# A/B of the tile factorisation's operand feed (scripts/traffic_ab.py): device time per launch
# as shipped (variant 0), with every update on the same 8 MB operand window (64), and with a
# cache-resident 1 KB feed (128); then FETCH_SIZE / WRITE_SIZE passes of each.
set -e
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out/ab
for v in ${AB_VARIANTS:-0 64 128 0 64 128}; do GPRX_PT_VARIANT=$v timeout -k 10 120 python3 scripts/traffic_ab.py >> gpurun_out/ab/ab.jsonl; done
cd /tmp
for v in ${AB_PMC:-128}; do
  export GPRX_PT_VARIANT=$v AB_ITERS=2
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/ab/f$v -o f -- python3 $R/scripts/traffic_ab.py > $R/gpurun_out/ab/f$v.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/ab/w$v -o w -- python3 $R/scripts/traffic_ab.py > $R/gpurun_out/ab/w$v.log 2>&1
done
echo done
