# (round 6 experiment: the shuffled records were slower and were removed; profiles/r06/ab_rec_shuffle/)
# SPL record loads per lane (the last one by shuffle): full GPU suite, then interleaved A/B against the
# previous library (variants/prev, a dev build of the parent commit) at C2, the N = 8 G = 1 share and the d split
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_tests.sh r06rec || exit 1
REPS=3 bash tools/gpu_ab.sh "c2prev|SM_LIB=variants/prev/libstereomst.so|" "c2new|SM_LIB=stereomatch_amd/libstereomst_dev.so|" \
  "s8prev|SM_LIB=variants/prev/libstereomst.so|--emulate-rank 0/8 --frame-groups 1" "s8new|SM_LIB=stereomatch_amd/libstereomst_dev.so|--emulate-rank 0/8 --frame-groups 1" \
  "d8prev|SM_LIB=variants/prev/libstereomst.so|--emulate-rank 0/8 --frame-groups 1 --shard d" "d8new|SM_LIB=stereomatch_amd/libstereomst_dev.so|--emulate-rank 0/8 --frame-groups 1 --shard d"
