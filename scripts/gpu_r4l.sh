set -e -o pipefail
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pack.py tests/test_gpu_dist.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 600 python -u scripts/config5_rank.py > $O/c5.json 2> $O/c5.err
python3 -c "import json;d=json.load(open('$O/c5.json'));print(d['ms_per_step'],d['ms_per_step_dense_exchange'],d['packed_exchange_ratio'],{k:(v['launches'],round(v['avg_ms'],3),round(v['gbs'])) for k,v in d['kernels'].items()}, {p:(round(c['step_ms_overlapped'],1),round(c['step_ms_overlapped_dense'],1)) for p,c in d['predicted_curve'].items()})"
