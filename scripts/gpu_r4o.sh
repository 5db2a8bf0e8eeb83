set -e -o pipefail
R=$PWD
O=$R/gpurun_out/r4o
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "gemm_tn" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 200 python -u scripts/bench_wide_gemm.py > $O/wgemm.json 2> $O/wgemm.err
head -1 $O/wgemm.json
for i in 1 2; do
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 > $O/c3_def_$i.json 2>/dev/null
  timeout -k 10 200 python -u scripts/bench_workloads.py --workload config3 --opt heavy_mid_side=1 > $O/c3_mid_$i.json 2>/dev/null
  python3 -c "import json;a=json.load(open('$O/c3_def_$i.json'));b=json.load(open('$O/c3_mid_$i.json'));print('default',round(a['ms_per_step'],3),round(a['host_issue_ms_per_step'],3),'mid_side',round(b['ms_per_step'],3),round(b['host_issue_ms_per_step'],3))"
done
