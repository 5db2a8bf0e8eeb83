set -e -o pipefail
# config 3: backward residual kernel at U = 4 gathers in flight per group
# (96 VGPRs, 5 waves; libmgcn_u4.so) vs U = 8 (107, 4 waves)
R=$PWD
O=$R/gpurun_out/r4u4
mkdir -p $O
MGCN_LIB=$R/meta-gcn_amd/mgcn/libmgcn_u4.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_residual.py tests/test_gpu_fullsize.py -k "residual or config3" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2 3; do
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_def_$i.json 2>/dev/null
  MGCN_LIB=$R/meta-gcn_amd/mgcn/libmgcn_u4.so timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_u4_$i.json 2>/dev/null
  python3 -c "import json;f=lambda t: round(json.load(open('$O/c3_%s_$i.json'%t))['ms_per_step'],3);print('def',f('def'),'u4',f('u4'))"
done
