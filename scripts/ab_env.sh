#!/bin/bash
# Headline bench A/B of an environment switch (repo root on the GPU box):
#   bash scripts/ab_env.sh <tag> <VAR> <value A> <value B> [tests...]
set -e -o pipefail
O=gpurun_out/$1; V=$2; A=$3; B=$4; shift 4
mkdir -p $O
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -q --timeout 150 --timeout-method thread \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for r in 1 2; do
  for x in $A $B; do
    env $V=$x timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-kernel-timers > $O/b.json 2>/dev/null
    python3 -c "import json;d=json.load(open('$O/b.json'));print('$V=$x', round(d['ms_per_step'],4))"
  done
done
