#!/bin/bash
# SQ counters of the config-3 step's kernels (wave cycles, waits, instruction
# mix), one rocprofv3 --pmc pass per counter group, each under its own limit
# (repo root on the GPU box):   bash scripts/prof_c3_sq.sh <tag>
set -e -o pipefail
R=$PWD
O=$R/gpurun_out/${1:?tag}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
W="python3 $R/scripts/bench_workloads.py --workload config3 --steps 3 --warmup 1"
i=0
for g in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d $O/pmc$i -o pmc -- $W > $O/pmc$i.log 2>&1 \
    || echo "pass $i failed: $g"
done
echo prof_c3_sq done
