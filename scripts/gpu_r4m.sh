set -e -o pipefail
O=gpurun_out/r4m
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "gemm_tn" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 200 python -u scripts/bench_wide_gemm.py > $O/wgemm.json 2> $O/wgemm.err
cat $O/wgemm.json
