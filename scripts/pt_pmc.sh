#!/bin/bash
# PMC passes over the tile-dataflow factorisation (devbench what=9, n=16384), one pass each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
rocprofv3 -L > $R/gpurun_out/pmc_list.txt 2>&1 || true
i=0
for ctrs in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_F64" "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d $R/gpurun_out/pmc$i -o p -- python3 $R/scripts/devbench_one.py 9 16384 > $R/gpurun_out/pmc$i.log 2>&1
  echo "pass $i rc=$?"
done
