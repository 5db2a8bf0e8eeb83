#!/bin/bash
# Profile pass of a round (run from the repo root on the GPU box):
#   bash scripts/profile_round.sh <tag>
# -> gpurun_out/<tag>/: the default bench.py line, a rocprofv3
# --kernel-trace --stats run of the same command, FETCH_SIZE / WRITE_SIZE PMC
# passes (one counter per run, no trace domains) over the config-2 layer
# kernels (scripts/prof_fused_once.py), and the known-byte calibration launch
# the PMC summary divides by (scripts/pmc_summary.py gpurun_out/<tag>
# profiles/<round>/pmc_fused.json).
# Every GPU step has its own limit; the chain stops at the first failure.
set -e -o pipefail
R=$PWD
T=${1:?tag}
O=$R/gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- \
  python3 $R/bench.py --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err
for k in fwd fwd_z bwd bwd_dw bwd_dx gemm_dw gemm_dw_cs; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${k}_$c -o pmc -- \
      python3 $R/scripts/prof_fused_once.py $k 3 > /dev/null 2>&1
  done
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_cal_FETCH_SIZE -o pmc -- \
  python3 $R/scripts/bench_spmm.py --calibrate > /dev/null 2>&1
echo profile_round $T done
