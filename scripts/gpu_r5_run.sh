set -e -o pipefail
O=gpurun_out/r5a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_guard.py tests/test_gpu_rccl.py tests/test_gpu_fused_wide.py tests/test_gpu_residual.py tests/test_gpu_dist.py tests/test_gpu_dp.py -x -v --timeout 240 --timeout-method thread > $O/t.log 2>&1 || { tail -60 $O/t.log; exit 1; }
tail -3 $O/t.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2>$O/bench.err
python3 scripts/ab_summary.py $O/bench.json bench
for i in 1 2; do
timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_$i.json 2>/dev/null
python3 scripts/ab_summary.py $O/c3_$i.json config3
done
timeout -k 10 400 python -u scripts/bench_wide.py --opts wide_pair=0 wide_pair=3 wide_pair=1 wide_pair=0,wide_unroll=8 > $O/wide.json 2>$O/wide.err || { tail -30 $O/wide.err; exit 1; }
cat $O/wide.err | grep opts
timeout -k 10 400 python -u scripts/config5_rank.py --steps 2 > $O/c5.json 2>$O/c5.err || { tail -30 $O/c5.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/c5.json'));print(d['ms_per_step'], d['ms_per_step_dense_exchange']); print(d['sampled_check']['worst'], d['sampled_check']['ok']); print({k:(round(v['avg_ms'],3), round(v['gbs'] or 0)) for k,v in d['kernels'].items()})"
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread > $O/tf.log 2>&1 || { tail -60 $O/tf.log; exit 1; }
tail -3 $O/tf.log
