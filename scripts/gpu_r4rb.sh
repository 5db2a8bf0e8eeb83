set -e -o pipefail
# config 3: workgroups per residual light-row launch (grid-stride beyond)
R=$PWD
O=$R/gpurun_out/r4rb
mkdir -p $O
run() {
  local t=$1; shift
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 "$@" > $O/c3_$t.json 2>/dev/null
  python3 -c "import json;print('$t', round(json.load(open('$O/c3_$t.json'))['ms_per_step'],3))"
}
for i in 1 2; do
  run def_$i
  run b1024_$i --opt residual_blocks=1024
  run b1536_$i --opt residual_blocks=1536
  run b2048_$i --opt residual_blocks=2048
  run b3072_$i --opt residual_blocks=3072
done
