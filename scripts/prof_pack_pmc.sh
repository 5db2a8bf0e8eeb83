#!/bin/bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE: one rocprofv3 --pmc pass each) of the
# pack kernels at a config-5 chunk (scripts/bench_pack.py, 1 rep) on the GPU
# box, repo root:   bash scripts/prof_pack_pmc.sh <tag>
set -e -o pipefail
R=$PWD
O=$R/gpurun_out/${1:?tag}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
W="python3 $R/scripts/bench_pack.py --reps 1"
i=0
for g in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d $O/pmc$i -o pmc -- $W > $O/pmc$i.log 2>&1 \
    || echo "pass $i failed: $g"
done
echo prof_pack_pmc done
