#!/bin/bash
# Parametrised A/B run on the GPU box (repo root), replacing the one-off
# per-experiment wrappers of earlier rounds:
#   TESTS="tests/test_gpu_x.py" TESTS_K="y or z" bash scripts/gpu_ab.sh <tag> <workload> <reps> "<arm 1>" "<arm 2>" ...
# workload: bench | config3 | config4 | config4max | config5rank | cmd:<command>
# an arm is a space-separated list of VAR=value settings ("" = defaults), e.g.
#   "MGCN_LIB=$PWD/meta-gcn_amd/mgcn/libmgcn_x.so"  (an alternative build)
#   "MGCN_Z_MIDDLE=1"                               (a host switch)
# Arms alternate within each repetition (same box, interleaved); every GPU
# step has its own time limit and the chain stops at the first failure.
set -e -o pipefail
O=$PWD/gpurun_out/$1; W=$2; N=$3; shift 3
mkdir -p "$O"
KARG=()
if [ -n "$TESTS_K" ]; then KARG=(-k "$TESTS_K"); fi
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS "${KARG[@]}" -x -q --timeout 150 --timeout-method thread \
    > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
  tail -1 "$O/tests.log"
fi
case $W in
  bench) cmd="python -u bench.py --no-cpu-baseline" ;;
  config3) cmd="python -u scripts/bench_workloads.py --workload config3" ;;
  config4) cmd="python -u scripts/bench_workloads.py --workload config4 --timers" ;;
  config4max) cmd="python -u scripts/bench_workloads.py --workload config4 --aggr max --timers" ;;
  config5rank) cmd="python -u scripts/config5_rank.py" ;;
  cmd:*) cmd="${W#cmd:}"; W=cmd ;;
  *) echo "unknown workload $W"; exit 2 ;;
esac
for r in $(seq 1 "$N"); do
  i=0
  for arm in "$@"; do
    i=$((i + 1))
    f="$O/${W}_a${i}_r${r}"
    env $arm timeout -k 10 500 $cmd > "$f.json" 2> "$f.err" || { tail -20 "$f.err"; exit 1; }
    python3 scripts/ab_summary.py "$f.json" "arm$i r$r [$arm]"
  done
done
