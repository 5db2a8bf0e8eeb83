#!/bin/bash
# Max-aggregation check: parity tests touching max, config-4 max step time and
# its rocprofv3 kernel stats.
set -e -o pipefail
R=$PWD
O=$R/gpurun_out/max
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "max_adjoint" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u scripts/bench_workloads.py --workload config4 --aggr max > $O/c4max.json
cat $O/c4max.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c4 -- \
  python3 $R/scripts/bench_workloads.py --workload config4 --aggr max --steps 5 > /dev/null 2>&1
python3 - <<PY
import csv
for x in list(csv.DictReader(open('$O/prof/c4_kernel_stats.csv')))[:8]:
    print(x['Name'][:70], x['Calls'], round(float(x['AverageNs'])/1e3,1))
PY
