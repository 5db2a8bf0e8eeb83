#!/bin/bash
# SQ counters of the 256-wide layer kernels gathering a dense vs a packed
# table (scripts/bench_packed.py at the config-5 rank's shape, 1 rep), one
# rocprofv3 --pmc pass per counter group (repo root on the GPU box):
#   bash scripts/prof_packed_sq.sh <tag>
set -e -o pipefail
R=$PWD
O=$R/gpurun_out/${1:?tag}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
W="python3 $R/scripts/bench_packed.py --reps 1"
i=0
for g in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $g --output-format csv -d $O/pmc$i -o pmc -- $W > $O/pmc$i.log 2>&1 \
    || echo "pass $i failed: $g"
done
echo prof_packed_sq done
