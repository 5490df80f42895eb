# One GPU session (edited per session; logs under gpurun_out/s/)
# This session: the chain kernels' helper waves at issue priority 1 (-DSM_CHAIN_HPRIO=1; chain waves stay
# at 3), C2 interleaved against the in-tree build, 4 reps, and the N = 8 share.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s
V=$GRAFT_REPO_ROOT/variants
REPS=4 bash tools/gpu_ab.sh "ch1|SM_LIB=$V/ch1/libstereomst.so|" "base||" || exit 3
REPS=1 bash tools/gpu_ab.sh "e8base||--emulate-rank 0/8 --frame-groups 1" "e8ch1|SM_LIB=$V/ch1/libstereomst.so|--emulate-rank 0/8 --frame-groups 1" || exit 4
