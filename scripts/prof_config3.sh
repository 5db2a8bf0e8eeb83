#!/bin/bash
# Config-3 profile (repo root on the GPU box): rocprofv3 kernel stats of the
# 12-layer botnet training step and a cProfile of its host issue.
#   bash scripts/prof_config3.sh <tag>
set -e -o pipefail
R=$PWD
O=$R/gpurun_out/${1:?tag}
mkdir -p $O
timeout -k 10 200 python -u scripts/prof_host_c3.py > $O/host_c3.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o c3 -- \
  python3 $R/scripts/bench_workloads.py --workload config3 > $O/config3_under_rocprof.json 2>&1
echo prof_config3 done
