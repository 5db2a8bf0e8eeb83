#!/bin/bash
# Round-end GPU pass: full GPU suite, smoke, default bench, config-3 kernel
# stats and the dense-GEMM PMC passes.  Every GPU step has its own limit and
# the chain stops at the first failure.
set -e -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c3 -o c3 -- \
  python3 $R/scripts/bench_workloads.py --workload config3 \
  > $R/gpurun_out/config3.json 2> $R/gpurun_out/config3.err
for k in nn bwd_relu bwd_dw; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pmc_${k}_$c -o pmc -- \
      python3 $R/scripts/prof_gemm_once.py $k 5 > /dev/null
  done
done
echo final_gpu done
