set -e -o pipefail
R=$PWD
O=$R/gpurun_out/r4s
mkdir -p $O
timeout -k 10 300 python -u scripts/bench_workloads.py --workload config4 --aggr max,add --timers > $O/config4_timers.json 2> $O/c4.err
cat $O/config4_timers.json
timeout -k 10 600 python -u scripts/config5_rank.py > $O/c5.json 2> $O/c5.err
python3 -c "import json;d=json.load(open('$O/c5.json'));print(d['ms_per_step'],d['ms_per_step_dense_exchange'],{k:(v['launches'],round(v['avg_ms'],3),round(v['gbs'])) for k,v in d['kernels'].items()}, {p:(round(c['step_ms_overlapped'],1),round(c['step_ms_overlapped_dense'],1)) for p,c in d['predicted_curve'].items()})"
bash scripts/prof_c3_pmc.sh r4s
