#!/bin/bash
# A/B of two library builds on the config-3 / config-4 workloads, interleaved:
#   bash scripts/ab_workloads.sh <libA> <libB> [bench_workloads args...]
set -e -o pipefail
A=$1; B=$2; shift 2
for i in 1 2; do
  for l in $A $B; do
    echo -n "$l: "
    MGCN_LIB=$l timeout -k 10 200 python -u scripts/bench_workloads.py "$@"
  done
done
