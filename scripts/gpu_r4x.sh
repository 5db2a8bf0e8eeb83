set -e -o pipefail
# non-giant heavy rows inside the residual light-row launch (libmgcn.so, option
# residual_mid_in_light 1 / 0) vs HEAD (libmgcn_head.so): residual / config-3
# tests, then a config-3 A/B
R=$PWD
O=$R/gpurun_out/r4x
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_residual.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_dp.py -k "residual or config3 or gcn_model or botnet" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2; do
  MGCN_LIB=$R/meta-gcn_amd/mgcn/libmgcn_head.so timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_head_$i.json 2>/dev/null
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_on_$i.json 2>/dev/null
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 --opt residual_mid_in_light=0 > $O/c3_off_$i.json 2>/dev/null
  python3 -c "import json;f=lambda t: round(json.load(open('$O/c3_%s_$i.json'%t))['ms_per_step'],3);print('head',f('head'),'on',f('on'),'off',f('off'))"
done
