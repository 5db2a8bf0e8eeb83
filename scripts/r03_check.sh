#!/bin/bash
# Round-3 GPU check: selected test files, smoke and the default bench.
# Usage (repo root on the GPU box): bash scripts/r03_check.sh <tag> <test files...>
set -e -o pipefail
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest "$@" -x -v --timeout 150 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
python3 -c "
import json;d=json.load(open('$O/bench.json'));print('bench', round(d['ms_per_step'],4), d['roofline']['frac'], {k:round(v['avg_ms'],4) for k,v in d['kernels'].items()})"
