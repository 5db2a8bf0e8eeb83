set -e -o pipefail
O=gpurun_out/${TAG:-r5max}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q -k "max_layer_with_next or max_stack_with" --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
for v in 1 0; do
MGCN_MAX_NEXT=$v timeout -k 10 300 python -u scripts/bench_workloads.py --workload config4 --aggr max --timers > $O/c4_$v.json 2>$O/c4_$v.err
python3 -c "
import json;d=json.load(open('$O/c4_$v.json'));v=d['max'];print('max_next=$v', round(v['ms_per_step'],3), {k:(x['launches'],round(x['avg_ms'],3)) for k,x in v.get('kernels',{}).items()})"
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -x -q -k "config4" --timeout 300 --timeout-method thread > $O/tf.log 2>&1 || { tail -40 $O/tf.log; exit 1; }
tail -2 $O/tf.log
