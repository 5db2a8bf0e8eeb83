set -e -o pipefail
O=gpurun_out/${TAG:-r5pool}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_kernel.py -x -q --timeout 200 --timeout-method thread > $O/t_pool.log 2>&1 || { tail -40 $O/t_pool.log; exit 1; }
tail -2 $O/t_pool.log
