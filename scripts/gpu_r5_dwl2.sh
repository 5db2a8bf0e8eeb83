set -e -o pipefail
O=gpurun_out/${TAG:-r5d}; mkdir -p $O
run() {  # tag, env, bench args
MGCN_DWL=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 ${@:3} > $O/bench_$1.json 2>$O/bench_$1.err
python3 -c "
import json;d=json.load(open('$O/bench_$1.json'));print('$1', round(d['ms_per_step'],3), {k:(v['launches'],round(v['avg_ms'],3)) for k,v in d['kernels'].items()})"
}
run dwl 1
run dbg1 1 --opt xw_ws_dbg=1
run dbg2 1 --opt xw_ws_dbg=2
run dbg4 1 --opt xw_ws_dbg=4
run dbg5 1 --opt xw_ws_dbg=5
