# Upper bound of a dependency-driven walker: the frame with the small walker rounds skipped (timing only,
# wrong results; dev library), C2 and the N = 8 G = 1 share, interleaved.
set -o pipefail
D="SM_LIB=stereomatch_amd/libstereomst_dev.so"
REPS=2 bash tools/gpu_ab.sh "c2base|$D|" "c2skip|$D SM_EXP_SKIP_SMALL_WALK=100000|" \
  "s8base|$D|--emulate-rank 0/8 --frame-groups 1" "s8skip|$D SM_EXP_SKIP_SMALL_WALK=100000|--emulate-rank 0/8 --frame-groups 1" \
  "s8base1|$D|--emulate-rank 0/8 --frame-groups 1 --inflight 1" "s8skip1|$D SM_EXP_SKIP_SMALL_WALK=100000|--emulate-rank 0/8 --frame-groups 1 --inflight 1"
