# Chain run window (SM_RUN_DIV: bucket nodes / div per run, dev builds) and piece length (SM_PIECE_LEN) at C2,
# interleaved against the defaults (div 384, P 512)
set -o pipefail
D="SM_LIB=stereomatch_amd/libstereomst_dev.so"
REPS=2 bash tools/gpu_ab.sh "base|$D|" "div256|$D SM_RUN_DIV=256|" "div512|$D SM_RUN_DIV=512|" "div768|$D SM_RUN_DIV=768|" \
  "p384|$D SM_PIECE_LEN=384|" "p640|$D SM_PIECE_LEN=640|"
