set -e -o pipefail
# config 3: split count of the staged weight GEMM (512 default, 768 / 256)
R=$PWD
O=$R/gpurun_out/r4sp
mkdir -p $O
for i in 1 2 3; do
  for v in def s768 s256; do
    if [ $v = def ]; then unset MGCN_LIB; else export MGCN_LIB=$R/meta-gcn_amd/mgcn/libmgcn_$v.so; fi
    timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_${v}_$i.json 2>/dev/null
  done
  unset MGCN_LIB
  python3 -c "import json;f=lambda t: round(json.load(open('$O/c3_%s_$i.json'%t))['ms_per_step'],3);print('def',f('def'),'s768',f('s768'),'s256',f('s256'))"
done
