set -e -o pipefail
O=gpurun_out/${TAG:-r5max}; mkdir -p $O
for u in 6 8 4; do
MGCN_MAX_NEXT=1 timeout -k 10 300 python -u scripts/bench_workloads.py --workload config4 --aggr max --timers --opt xw_ws_xm_unroll=$u > $O/c4_u$u.json 2>$O/c4_u$u.err
python3 -c "
import json;d=json.load(open('$O/c4_u$u.json'));v=d['max'];print('u=$u', round(v['ms_per_step'],3), {k:(x['launches'],round(x['avg_ms'],3)) for k,x in v.get('kernels',{}).items()})"
done
