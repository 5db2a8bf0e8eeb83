# F = 256 kernels: parity tests (both forms), then config 5's rank-local step
set -e -o pipefail
O=gpurun_out/${TAG:-r5c5}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_wide.py tests/test_gpu_guard.py -x -q --timeout 200 --timeout-method thread > $O/t_wide.log 2>&1 || { tail -60 $O/t_wide.log; exit 1; }
tail -2 $O/t_wide.log
timeout -k 10 500 python -u scripts/config5_rank.py --steps 2 > $O/c5.json 2>$O/c5.err || { tail -30 $O/c5.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/c5.json'));print(d['ms_per_step'], d.get('ms_per_step_dense_exchange')); print(d.get('sampled_check')); print({k:(round(v['avg_ms'],3), round(v['gbs'] or 0)) for k,v in d['kernels'].items()})"
