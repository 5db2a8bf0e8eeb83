set -e -o pipefail
R=$PWD
O=$R/gpurun_out/r4t
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/def_$i.json 2>/dev/null
  MGCN_LIB=$R/meta-gcn_amd/mgcn/libmgcn_nt2.so timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/nt2_$i.json 2>/dev/null
  python3 -c "
import json
for t in ('def','nt2'):
    d=json.load(open('$O/%s_$i.json'%t)); print(t, round(d['ms_per_step'],4), {k:round(v['avg_ms'],4) for k,v in d['kernels'].items()})"
done
