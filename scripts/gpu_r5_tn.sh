set -e -o pipefail
O=gpurun_out/${TAG:-r5tn}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_wide.py -x -q -k "stack" --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
for o in gemm_tn_wide2=0 gemm_tn_wide2=1 gemm_tn_wide2=0 gemm_tn_wide2=1; do
timeout -k 10 200 python -u scripts/bench_wide_gemm.py --opt $o > $O/tn_$o.json 2>$O/tn_$o.err
python3 -c "import json;d=json.loads(open('$O/tn_$o.json').readline());print('$o', round(d['ms'],3), round(d['gbs']), d['err'])"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_pool.py -x -q --timeout 200 --timeout-method thread > $O/t_pool.log 2>&1 || { tail -40 $O/t_pool.log; exit 1; }
tail -2 $O/t_pool.log
