set -e -o pipefail
# the GPU suite on the heavy.h refactor (libmgcn.so), then config-3 A/B
# against HEAD (libmgcn_head.so), the new library first in each pair
R=$PWD
O=$R/gpurun_out/r4y
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for i in 1 2 3; do
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_new_$i.json 2>/dev/null
  MGCN_LIB=$R/meta-gcn_amd/mgcn/libmgcn_head.so timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_head_$i.json 2>/dev/null
  python3 -c "import json;f=lambda t: round(json.load(open('$O/c3_%s_$i.json'%t))['ms_per_step'],3);print('new',f('new'),'head',f('head'))"
done
