#!/bin/bash
# Config-3 roofline passes (repo root on the GPU box): a kernel trace and three
# PMC passes (L2 hit / miss, FETCH_SIZE, WRITE_SIZE; one TCC group per run, no
# trace domains) of the config-3 step, summarised by scripts/c3_roofline.py.
#   bash scripts/prof_c3_pmc.sh <tag>
set -e -o pipefail
R=$PWD
O=$R/gpurun_out/${1:?tag}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
W="python3 $R/scripts/bench_workloads.py --workload config3 --steps 3 --warmup 1"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/c3_trace -o c3 -- $W > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/c3_hit -o pmc -- $W > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c3_fetch -o pmc -- $W > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c3_write -o pmc -- $W > /dev/null 2>&1
cd $R
python3 scripts/c3_roofline.py $O/c3_trace $O/c3_hit $O/c3_fetch $O/c3_write $O/config3_roofline.json
echo prof_c3_pmc done
