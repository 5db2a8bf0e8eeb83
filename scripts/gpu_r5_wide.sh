# A/B of the F = 256 layer kernel forms (scripts/bench_wide.py), args = --opts list
set -e -o pipefail
O=gpurun_out/${TAG:-r5w}; mkdir -p $O
timeout -k 10 500 python -u scripts/bench_wide.py --opts "$@" > $O/wide.json 2>$O/wide.err || { tail -30 $O/wide.err; exit 1; }
grep opts $O/wide.err
python -c "import json; d=json.load(open('$O/wide.json')); print('spmm_fwd', d['spmm_fwd'])"
