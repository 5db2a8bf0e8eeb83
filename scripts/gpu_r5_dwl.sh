# F = 128 warp-specialised adjoint + fused lower dW: parity, then the bench A/B
set -e -o pipefail
O=gpurun_out/${TAG:-r5d}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_ws.py -x -q --timeout 200 --timeout-method thread > $O/t_ws.log 2>&1 || { tail -60 $O/t_ws.log; exit 1; }
tail -2 $O/t_ws.log
run() {  # tag, env, bench args
MGCN_DWL=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline ${@:3} > $O/bench_$1.json 2>$O/bench_$1.err
python3 -c "
import json;d=json.load(open('$O/bench_$1.json'));print('$1', round(d['ms_per_step'],3), {k:(v['launches'],round(v['avg_ms'],3)) for k,v in d['kernels'].items()})"
}
run dwl 1
run ws_dx 0
run legacy_dx 0 --opt xw_ws=0
run dwl_u8 1 --opt xw_ws_unroll=8
