#!/bin/bash
# End-of-round GPU pass (repo root on the GPU box): the GPU suite, smoke,
# profile_round.sh (bench line, rocprofv3 stats, PMC passes), the config-3 /
# config-4 workloads and config 3's kernel stats.  bash scripts/round_final.sh <tag>
set -e -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
bash scripts/profile_round.sh $T
timeout -k 10 300 python -u scripts/bench_workloads.py --workload config3 > $O/config3.json 2>/dev/null
timeout -k 10 300 python -u scripts/bench_workloads.py --workload config4 > $O/config4.json 2>/dev/null
cat $O/config3.json $O/config4.json
bash scripts/kstats_c3.sh $T/c3 meta-gcn_amd/mgcn/libmgcn.so > /dev/null
echo round_final done
