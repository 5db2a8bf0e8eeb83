#!/bin/bash
# gpu_check.sh without -x: every GPU test runs (the list of failures, not the first); then smoke, the bench, the
# config-3/4 workloads and a rocprofv3 --kernel-trace --stats run of the bench.
# Usage (repo root on the GPU box): bash scripts/gpu_check.sh <tag> [pytest -k expr]
# Every GPU step has its own limit; the chain stops at the first failure.
set -e -o pipefail
R=$PWD
T=${1:-dev}
O=$R/gpurun_out/$T
mkdir -p $O
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -k "$K" \
    > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
    > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
fi
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
python3 -c "
import json;d=json.load(open('$O/bench_default.json'));print('bench', round(d['ms_per_step'],4), {k:round(v['avg_ms'],4) for k,v in d['kernels'].items()})"
timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/config3.json
timeout -k 10 300 python -u scripts/bench_workloads.py --workload config4 > $O/config4.json
cat $O/config3.json $O/config4.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- \
  python3 $R/bench.py --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o c3 -- \
  python3 $R/scripts/bench_workloads.py --workload config3 > /dev/null 2>&1
echo gpu_check $T done
