#!/bin/bash
# Bench experiment builds: scripts/variant_bench.sh "<lib or ->|<MGCN_OPTIONS>" ...
# Prints ms/step and per-kernel averages for each (lib, options) pair.
set -e -o pipefail
mkdir -p gpurun_out/var
i=0
for spec in "$@"; do
  i=$((i+1))
  lib=${spec%%|*}; opt=${spec#*|}
  [ "$lib" = "-" ] && lib=""
  MGCN_LIB=$lib MGCN_OPTIONS=$opt timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/var/b$i.json
  python3 -c "
import json,sys;d=json.load(open('gpurun_out/var/b$i.json'));print(sys.argv[1], round(d['ms_per_step'],4), {k:round(v['avg_ms'],4) for k,v in d['kernels'].items()})" "$spec"
done
