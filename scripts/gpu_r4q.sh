set -e -o pipefail
# config 3: edge quads in flight per producer in the non-giant heavy-row
# workgroups, 4 (default) vs 2 / 1 (libmgcn_q2.so / libmgcn_q1.so)
R=$PWD
O=$R/gpurun_out/r4q
mkdir -p $O
for i in 1 2 3; do
  for v in def q2 q1; do
    if [ $v = def ]; then unset MGCN_LIB; else export MGCN_LIB=$R/meta-gcn_amd/mgcn/libmgcn_$v.so; fi
    timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_${v}_$i.json 2>/dev/null
  done
  unset MGCN_LIB
  python3 -c "import json;f=lambda t: round(json.load(open('$O/c3_%s_$i.json'%t))['ms_per_step'],3);print('def',f('def'),'q2',f('q2'),'q1',f('q1'))"
done
