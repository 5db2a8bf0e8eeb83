set -e -o pipefail
# config 4 max: GEMM outputs nt vs default policy (libmgcn_gnont.so), SpMM unroll
R=$PWD
O=$R/gpurun_out/r4c4
mkdir -p $O
run() {  # tag, env lib or '', options...
  local t=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then export MGCN_LIB=$R/meta-gcn_amd/mgcn/$lib; else unset MGCN_LIB; fi
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config4 --aggr max --timers "$@" > $O/c4_$t.json 2>/dev/null
  unset MGCN_LIB
  python3 -c "
import json; d=json.load(open('$O/c4_$t.json'))['max']; print('$t', round(d['ms_per_step'],3), {k:round(v['avg_ms'],3) for k,v in d['kernels'].items()})"
}
for i in 1 2; do
  run def_$i ''
  run gnont_$i libmgcn_gnont.so
  run u4_$i '' --opt spmm_unroll=4
  run u16_$i '' --opt spmm_unroll=16
done
