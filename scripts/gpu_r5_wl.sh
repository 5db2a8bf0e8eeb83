# config 3 / config 4 workloads (scripts/bench_workloads.py) + config-3 full-size parity
set -e -o pipefail
O=gpurun_out/${TAG:-r5wl}; mkdir -p $O
for i in 1 2; do
timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_$i.json 2>$O/c3_$i.err
python3 -c "import json;d=json.load(open('$O/c3_$i.json'));print('config3', {k:v for k,v in d.items() if 'ms' in k or 'host' in k})"
done
timeout -k 10 300 python -u scripts/bench_workloads.py --workload config4 --timers > $O/c4.json 2>$O/c4.err
python3 -c "
import json;d=json.load(open('$O/c4.json'))
for a in ('add','mean','max'):
  v=d.get(a)
  if v: print(a, round(v['ms_per_step'],3), {k:(x['launches'],round(x['avg_ms'],3)) for k,x in v.get('kernels',{}).items()})"
timeout -k 10 300 python -u -m pytest tests/test_gpu_pack.py tests/test_gpu_dist.py tests/test_gpu_rccl.py tests/test_gpu_guard.py -x -q --timeout 200 --timeout-method thread > $O/t_pack.log 2>&1 || { tail -40 $O/t_pack.log; exit 1; }
tail -2 $O/t_pack.log
timeout -k 10 500 python -u scripts/config5_rank.py --steps 2 > $O/c5.json 2>$O/c5.err || { tail -30 $O/c5.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/c5.json'));print(d['ms_per_step'], d.get('ms_per_step_dense_exchange')); print(d['sampled_check']['worst'], d['sampled_check']['ok']); print({k:(round(v['avg_ms'],3), round(v['gbs'] or 0)) for k,v in d['kernels'].items()})"
