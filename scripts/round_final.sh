#!/bin/bash
# End-of-round GPU pass (repo root on the GPU box): the GPU suite and smoke
# (round_final_tests.sh), then profile_round.sh (bench line, rocprofv3
# stats, PMC passes) and the config-3 / config-4 workloads
# (round_final_profile.sh).  Each half also runs as its own gpurun call when
# the two together would pass gpurun's time limit.
#   bash scripts/round_final.sh <tag>
set -e -o pipefail
T=${1:?tag}
bash scripts/round_final_tests.sh $T
bash scripts/round_final_profile.sh $T
echo round_final done
