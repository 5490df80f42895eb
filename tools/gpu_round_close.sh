# Close of round 3: PMS parity + dedupe A/B, the full final check, then the profile set of this build
set -o pipefail
bash tools/gpu_pms_ab.sh || exit 1
bash tools/gpu_final.sh || exit 2
bash tools/gpu_prof_round.sh r03c || exit 3
