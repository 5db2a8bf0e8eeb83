#!/bin/bash
# rocprofv3 kernel stats of config 3 for each given libmgcn build (repo root on the GPU box):
#   bash scripts/kstats_c3.sh <tag> <lib>...
set -e -o pipefail
R=$PWD; O=$R/gpurun_out/$1; shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for L in "$@"; do
  MGCN_LIB=$R/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$i -o c3 -- \
    python3 $R/scripts/bench_workloads.py --workload config3 --steps 10 > $O/p$i.log 2>&1
  echo "== $L"
  python3 - $(find $O/p$i -name '*kernel_stats.csv' | head -1) <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:9]:
    print(r['Calls'], round(float(r['AverageNs']) / 1e3, 1), round(float(r['TotalDurationNs']) / 1e6, 2), r['Name'][:80])
PY
  i=$((i+1))
done
