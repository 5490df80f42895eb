# One GPU session (edited per session; logs under gpurun_out/s/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s
REPS=2 bash tools/gpu_ab.sh "new||" "uns5|SM_LIB=$GRAFT_REPO_ROOT/variants/uns5/libstereomst.so|" "uns6|SM_LIB=$GRAFT_REPO_ROOT/variants/uns6/libstereomst.so|" || exit 4
