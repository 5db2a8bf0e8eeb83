# Profile pass + config-3 / config-4 workloads: the second half of
# scripts/round_final.sh, as its own gpurun call
#   bash scripts/round_final_profile.sh <tag>
set -e -o pipefail
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
bash scripts/profile_round.sh $T
timeout -k 10 300 python -u scripts/bench_workloads.py --workload config3 > $O/config3.json 2>/dev/null
timeout -k 10 300 python -u scripts/bench_workloads.py --workload config4 > $O/config4.json 2>/dev/null
echo final_b done
