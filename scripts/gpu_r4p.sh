set -e -o pipefail
# config 3: workgroup cap of the backward light-row launch (its column-sum
# partial slots): 2048 (default) vs 4096 / 8192 (libmgcn_p4096 / p8192)
R=$PWD
O=$R/gpurun_out/r4p
mkdir -p $O
MGCN_LIB=$R/meta-gcn_amd/mgcn/libmgcn_p8192.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_residual.py tests/test_gpu_fullsize.py -k "residual or config3" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2 3; do
  for v in def p4096 p8192; do
    if [ $v = def ]; then unset MGCN_LIB; else export MGCN_LIB=$R/meta-gcn_amd/mgcn/libmgcn_$v.so; fi
    timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_${v}_$i.json 2>/dev/null
  done
  unset MGCN_LIB
  python3 -c "import json;f=lambda t: round(json.load(open('$O/c3_%s_$i.json'%t))['ms_per_step'],3);print('def',f('def'),'p4096',f('p4096'),'p8192',f('p8192'))"
done
