set -e -o pipefail
O=gpurun_out/${TAG:-r5dw}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_ws.py -x -q -k "dw_pass_ws" --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
run() {
MGCN_DWL=$2 MGCN_Z_MIDDLE=$3 timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 ${@:4} > $O/bench_$1.json 2>$O/bench_$1.err
python3 -c "
import json;d=json.load(open('$O/bench_$1.json'));print('$1', round(d['ms_per_step'],3), {k:(v['launches'],round(v['avg_ms'],3)) for k,v in d['kernels'].items()})"
}
run base 0 0 --opt xw_ws=0 --opt dw_ws=0
run dwws 0 0 --opt xw_ws=0
run dwws_zmid 0 1 --opt xw_ws=0
run dwws_zmid_xws 0 1
