set -e -o pipefail
# config 3: giant-row LDS / block and mid-heavy LDS sweep
R=$PWD
O=$R/gpurun_out/r4t3
mkdir -p $O
run() {  # tag, options...
  local t=$1; shift
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 "$@" > $O/c3_$t.json 2>/dev/null
  python3 -c "import json;print('$t', round(json.load(open('$O/c3_$t.json'))['ms_per_step'],3))"
}
for i in 1 2; do
  run def_$i
  run g128_$i --opt heavy_lds_kb=128
  run g96_$i --opt heavy_lds_kb=96
  run g64_$i --opt heavy_lds_kb=64
  run g96b512_$i --opt heavy_lds_kb=96 --opt heavy_block=512
  run m24_$i --opt heavy_mid_lds_kb=24
  run m64_$i --opt heavy_mid_lds_kb=64
  run gt1024_$i --opt heavy_giant_thr=1024
done
