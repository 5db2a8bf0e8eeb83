set -e -o pipefail
# restrict-LDS bodies for the fused and residual kernels (libmgcn.so) vs
# HEAD (libmgcn_pre.so): fused / residual tests, then config-2 and config-3 A/B
R=$PWD
O=$R/gpurun_out/r4r
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_headline.py tests/test_gpu_residual.py tests/test_gpu_fullsize.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/b_new_$i.json 2>/dev/null
  MGCN_LIB=$R/meta-gcn_amd/mgcn/libmgcn_pre.so timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/b_pre_$i.json 2>/dev/null
  python3 -c "
import json
for t in ('new','pre'):
    d=json.load(open('$O/b_%s_$i.json'%t)); print(t, round(d['ms_per_step'],4), {k:round(v['avg_ms'],4) for k,v in d['kernels'].items()})"
done
for i in 1 2; do
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_new_$i.json 2>/dev/null
  MGCN_LIB=$R/meta-gcn_amd/mgcn/libmgcn_pre.so timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_pre_$i.json 2>/dev/null
  python3 -c "import json;f=lambda t: round(json.load(open('$O/c3_%s_$i.json'%t))['ms_per_step'],3);print('c3 new',f('new'),'pre',f('pre'))"
done
