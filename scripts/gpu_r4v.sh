set -e -o pipefail
# residual forward transform in the heavy-row epilogue (libmgcn_epi.so) vs HEAD
# (libmgcn.so): its residual / config-3 tests, then a config-3 A/B; the config-4
# nt3 A/B (gpu_r4u.sh)
R=$PWD
O=$R/gpurun_out/r4v
mkdir -p $O
E=$R/meta-gcn_amd/mgcn/libmgcn_epi.so
MGCN_LIB=$E timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_residual.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "residual or config3" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2; do
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_old_$i.json 2>/dev/null
  MGCN_LIB=$E timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_new_$i.json 2>/dev/null
  python3 -c "import json;a=json.load(open('$O/c3_old_$i.json'));b=json.load(open('$O/c3_new_$i.json'));print('old',round(a['ms_per_step'],3),'new',round(b['ms_per_step'],3))"
done
bash scripts/gpu_r4u.sh
