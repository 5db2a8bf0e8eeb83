#!/bin/bash
# PMC passes over the fused kernels (one counter set per rocprofv3 run)
R=$PWD
mkdir -p gpurun_out/pmcf
cd /tmp && export TMPDIR=/tmp
for k in bwd bwd_dw fwd spmm; do
  i=0
  for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pmcf/${k}_$i -o pmc -- python3 $R/scripts/prof_fused_once.py $k 3 > /dev/null 2>&1 || { echo "pass $k $i failed"; exit 1; }
  done
done
echo pmc done
