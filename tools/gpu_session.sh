# One GPU session (edited per session; logs under gpurun_out/s/)
# This session: confirmation of the walkers' issue priority 1 (-DSM_WALK_PRIO=1), C2 interleaved, 4 reps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s
V=$GRAFT_REPO_ROOT/variants
REPS=4 bash tools/gpu_ab.sh "wp1|SM_LIB=$V/wp1/libstereomst.so|" "base||" || exit 3
