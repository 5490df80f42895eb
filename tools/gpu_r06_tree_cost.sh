# What the tree stages cost with frames in flight (dev library, timing only): C2 as is, re-filtering the previous
# layout (no prep / MST / layout), keeping the previous MST (prep + layout + filter), keeping the previous
# layout (prep + MST + filter); interleaved
set -o pipefail
D="SM_LIB=stereomatch_amd/libstereomst_dev.so"
REPS=2 bash tools/gpu_ab.sh "base|$D|" "filteronly|$D SM_EXP_FILTER_ONLY=1|" "skipmst|$D SM_EXP_SKIP=mst|" "skiplayout|$D SM_EXP_SKIP=layout|"
