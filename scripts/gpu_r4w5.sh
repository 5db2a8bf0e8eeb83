set -e -o pipefail
# residual tests on the default build; config-3 A/B: backward residual kernel
# at 4 waves (default, 107 VGPRs) vs 5 waves (libmgcn_w5.so, 96 VGPRs + spills)
R=$PWD
O=$R/gpurun_out/r4w5
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_residual.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "residual or config3 or gcn_model" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2; do
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_def_$i.json 2>/dev/null
  MGCN_LIB=$R/meta-gcn_amd/mgcn/libmgcn_w5.so timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_w5_$i.json 2>/dev/null
  python3 -c "import json;f=lambda t: round(json.load(open('$O/c3_%s_$i.json'%t))['ms_per_step'],3);print('def',f('def'),'w5',f('w5'))"
done
