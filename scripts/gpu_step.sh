#!/bin/bash
# Run one GPU step under its own time limit; stop the chain on a crash,
# fault, abort or timeout (exit codes other than 0 / 1 -- pytest's "tests
# failed" is 1 and does not end the chain).
# usage: bash scripts/gpu_step.sh <seconds> <log> <cmd...>
t=$1; log=$2; shift 2
timeout -k 10 "$t" "$@" > "$log" 2>&1
rc=$?
tail -15 "$log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STEP FAILED rc=$rc: $*"; exit $rc; fi
exit 0
