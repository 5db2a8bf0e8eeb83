#!/bin/bash
# Counters of the 256 x 256 dW (gemm_tn_x6_wide_kernel) at the config-5 rank
# shape (K = 6.24M): one rocprofv3 --pmc pass per counter group, each under its
# own time limit (run from the repo root on the GPU box):
#   bash scripts/prof_wide_gemm.sh <tag>
set -e -o pipefail
R=$PWD
O=$R/gpurun_out/${1:?tag}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for g in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA" \
         "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
         "FETCH_SIZE" "SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_VALU_MFMA_COEXEC_CYCLES"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $g --output-format csv -d $O/pmc$i -o pmc -- \
    python3 $R/scripts/bench_wide_gemm.py --tn-only > $O/pmc$i.log 2>&1 || echo "pass $i failed: $g"
done
echo prof_wide_gemm done
