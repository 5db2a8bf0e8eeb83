set -e -o pipefail
# config-4 A/B: HEAD vs the nt3 experiment build (SpMM / GEMM outputs nt)
R=$PWD
O=$R/gpurun_out/r4v
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python -u scripts/bench_workloads.py --workload config4 --timers > $O/def_$i.json 2>/dev/null
  MGCN_LIB=$R/meta-gcn_amd/mgcn/libmgcn_nt3.so timeout -k 10 300 python -u scripts/bench_workloads.py --workload config4 --timers > $O/nt3_$i.json 2>/dev/null
  python3 -c "
import json
for t in ('def','nt3'):
    d=json.load(open('$O/%s_$i.json'%t)); print(t, {a:round(d[a]['ms_per_step'],3) for a in ('add','mean','max')}, {k:round(v['avg_ms'],3) for k,v in d['max']['kernels'].items()})"
done
timeout -k 10 300 python -u scripts/prof_host_c3.py > $O/host_c3.txt 2>&1
head -60 $O/host_c3.txt
