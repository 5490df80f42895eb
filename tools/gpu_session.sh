# One GPU session (edited per session; logs under gpurun_out/s/)
# This session: frames in flight 3 (default) against 4 with the walkers at issue priority 1, C2 interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s
REPS=3 bash tools/gpu_ab.sh "if3||" "if4||--inflight 4" || exit 3
