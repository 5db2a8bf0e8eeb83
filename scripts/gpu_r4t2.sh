set -e -o pipefail
# config 3: heavy-row threshold sweep
R=$PWD
O=$R/gpurun_out/r4t2
mkdir -p $O
for i in 1 2; do
  for t in 128 96 192 256 384; do
    timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 --heavy-thr $t > $O/c3_${t}_$i.json 2>/dev/null
    python3 -c "import json;print($t, round(json.load(open('$O/c3_${t}_$i.json'))['ms_per_step'],3))"
  done
done
