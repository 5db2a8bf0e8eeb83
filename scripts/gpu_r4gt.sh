set -e -o pipefail
# config 3: giant-row threshold with the one-quad mid-heavy kernel
R=$PWD
O=$R/gpurun_out/r4gt
mkdir -p $O
run() {
  local t=$1; shift
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 "$@" > $O/c3_$t.json 2>/dev/null
  python3 -c "import json;print('$t', round(json.load(open('$O/c3_$t.json'))['ms_per_step'],3))"
}
for i in 1 2; do
  run def_$i
  run g256_$i --opt heavy_giant_thr=256
  run g384_$i --opt heavy_giant_thr=384
  run g768_$i --opt heavy_giant_thr=768
done
