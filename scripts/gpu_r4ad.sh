set -e -o pipefail
# config 3: torch Adam foreach (default) vs fused
R=$PWD
O=$R/gpurun_out/r4ad
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_def_$i.json 2>/dev/null
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 --adam fused > $O/c3_fused_$i.json 2>/dev/null
  python3 -c "import json;f=lambda t: json.load(open('$O/c3_%s_$i.json'%t));a=f('def');b=f('fused');print('def',round(a['ms_per_step'],3),round(a['host_issue_ms_per_step'],3),'fused',round(b['ms_per_step'],3),round(b['host_issue_ms_per_step'],3))"
done
