# (round 6 experiment: within noise, not kept; profiles/r06/ab_lr3/)
# Three light rows per up-walker chunk (SPL <= 2, 8-wave bound): full GPU suite, then interleaved A/B against the
# previous library (variants/prev, a dev build of the parent commit)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_tests.sh r06lr3 || exit 1
REPS=4 bash tools/gpu_ab.sh "c2prev|SM_LIB=variants/prev/libstereomst.so|" "c2lr3|SM_LIB=stereomatch_amd/libstereomst_dev.so|"
