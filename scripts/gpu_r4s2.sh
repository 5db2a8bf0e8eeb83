set -e -o pipefail
# config 3: the non-giant heavy rows on a second side stream (heavy_side_stream
# = 2) vs the default; residual tests with the option set
R=$PWD
O=$R/gpurun_out/r4s2
mkdir -p $O
MGCN_OPTIONS=heavy_side_stream=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_residual.py tests/test_gpu_fullsize.py -k "residual or config3" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2 3; do
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_def_$i.json 2>/dev/null
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 --opt heavy_side_stream=2 > $O/c3_s2_$i.json 2>/dev/null
  python3 -c "import json;f=lambda t: round(json.load(open('$O/c3_%s_$i.json'%t))['ms_per_step'],3);print('def',f('def'),'s2',f('s2'))"
done
