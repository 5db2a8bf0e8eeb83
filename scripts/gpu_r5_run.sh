# Round-5 GPU pass: the new wide kernels first (tests + A/B), the guard /
# RCCL tests, then the whole GPU suite and the bench.
set -e -o pipefail
O=gpurun_out/${1:-r5a}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_wide.py -x -v --timeout 200 --timeout-method thread > $O/t_wide.log 2>&1 || { tail -60 $O/t_wide.log; exit 1; }
tail -3 $O/t_wide.log
timeout -k 10 400 python -u scripts/bench_wide.py --opts wide_ws=0 wide_ws=3 wide_ws=3,wide_unroll=8 > $O/wide.json 2>$O/wide.err || { tail -30 $O/wide.err; exit 1; }
grep opts $O/wide.err
timeout -k 10 300 python -u -m pytest tests/test_gpu_guard.py tests/test_gpu_rccl.py -x -v --timeout 120 --timeout-method thread > $O/t_new.log 2>&1 || { tail -60 $O/t_new.log; exit 1; }
tail -3 $O/t_new.log
timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread --ignore=tests/test_gpu_guard.py --ignore=tests/test_gpu_rccl.py --ignore=tests/test_gpu_fused_wide.py > $O/t_all.log 2>&1 || { tail -60 $O/t_all.log; exit 1; }
tail -3 $O/t_all.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2>$O/bench.err
cat $O/bench.json
