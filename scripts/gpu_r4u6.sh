set -e -o pipefail
# config 4 max: SpMM unroll 6 for every mode (the max forward already runs 6)
R=$PWD
O=$R/gpurun_out/r4u6
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config4 --aggr max --timers > $O/def_$i.json 2>/dev/null
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config4 --aggr max --timers --opt spmm_unroll=6 > $O/u6_$i.json 2>/dev/null
  python3 -c "
import json
for t in ('def','u6'):
    d=json.load(open('$O/%s_$i.json'%t))['max']; print(t, round(d['ms_per_step'],3), {k:round(v['avg_ms'],3) for k,v in d['kernels'].items()})"
done
