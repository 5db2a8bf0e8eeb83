set -e -o pipefail
# residual backward: heavy rows' transform in the heavy-row epilogue + the
# weight GEMM riding in the next layer's light launch (libmgcn_bwd.so) vs HEAD
R=$PWD
O=$R/gpurun_out/r4w
mkdir -p $O
E=$R/meta-gcn_amd/mgcn/libmgcn_bwd.so
MGCN_LIB=$E timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_residual.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_dp.py -k "residual or config3 or gcn_model or botnet" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2; do
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_old_$i.json 2>/dev/null
  MGCN_LIB=$E timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_new_$i.json 2>/dev/null
  python3 -c "import json;a=json.load(open('$O/c3_old_$i.json'));b=json.load(open('$O/c3_new_$i.json'));print('old',round(a['ms_per_step'],3),'new',round(b['ms_per_step'],3))"
done
