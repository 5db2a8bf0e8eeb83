#!/bin/bash
# One rocprofv3 PMC pass per call: scripts/pmc_pass.sh OUTDIR "COUNTERS" -- python3 script args
set -e
out=$1; ctrs=$2; shift 3
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d "$out" -o pmc -- "$@"
