#!/bin/bash
# Config-3 option sweep (repo root on the GPU box): each line = libmgcn options
# for scripts/bench_workloads.py --workload config3.  Usage: bash scripts/sweep_c3.sh <tag> "<opts>" ...
set -e -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
i=0
for cfg in "$@"; do
  args=""
  for kv in $cfg; do args="$args --opt $kv"; done
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 $args > $O/c3_$i.json 2>/dev/null
  python3 -c "import json;d=json.load(open('$O/c3_$i.json'));print('$cfg', round(d['ms_per_step'],3), round(d['host_issue_ms_per_step'],3))"
  i=$((i+1))
done
