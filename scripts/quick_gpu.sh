set -e -o pipefail
mkdir -p gpurun_out/q
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/q/tests.log 2>&1 || { tail -30 gpurun_out/q/tests.log; exit 1; }
tail -2 gpurun_out/q/tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/q/bench.json
python3 -c "
import json;d=json.load(open('gpurun_out/q/bench.json'));print(d['ms_per_step']);print({k:round(v['avg_ms'],4) for k,v in d['kernels'].items()})"
