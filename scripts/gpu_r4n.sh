set -e -o pipefail
R=$PWD
O=$R/gpurun_out/r4n
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "gemm_tn" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 200 python -u scripts/bench_wide_gemm.py > $O/wgemm.json 2> $O/wgemm.err
cat $O/wgemm.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c3trace -o c3 -- \
  python3 $R/scripts/bench_workloads.py --workload config3 --steps 6 --warmup 2 > $O/c3.json 2> $O/c3.err
cd $R
python3 scripts/c3_timeline.py $O/c3trace > $O/c3_timeline.txt
head -3 $O/c3_timeline.txt
