set -e -o pipefail
# one edge quad in flight for narrow heavy rows (default now): heavy-row /
# residual tests, then config 3 vs heavy_mid_q1=0 and a mid-LDS sweep
R=$PWD
O=$R/gpurun_out/r4q2
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_residual.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_pool.py -k "heavy or skew or residual or config3 or star or pool" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
run() {
  local t=$1; shift
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 "$@" > $O/c3_$t.json 2>/dev/null
  python3 -c "import json;print('$t', round(json.load(open('$O/c3_$t.json'))['ms_per_step'],3))"
}
for i in 1 2; do
  run def_$i
  run q4_$i --opt heavy_mid_q1=0
  run m24_$i --opt heavy_mid_lds_kb=24
  run m32_$i --opt heavy_mid_lds_kb=32
  run m48_$i --opt heavy_mid_lds_kb=48
  run m64_$i --opt heavy_mid_lds_kb=64
done
