# One GPU session (edited per session; logs under gpurun_out/s/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "mst_ or timeout or layout or match_bitexact_golden or full_size_c2_match or pieces_match or full_size_c3_match" -x -v --timeout 300 --timeout-method thread > gpurun_out/s/tests.log 2>&1; rc=$?; tail -3 gpurun_out/s/tests.log; [ $rc -eq 0 ] || exit 3
REPS=2 bash tools/gpu_ab.sh "prev|SM_LIB=$GRAFT_REPO_ROOT/variants/prev/libstereomst.so|" "new||" || exit 4
REPS=2 BASE_ARGS="--emulate-rank 0/8 --frame-groups 1 --steps 20 --warmup 5 --no-cpu --no-host-io --no-pms --no-segment" bash tools/gpu_ab.sh "e_new||" "e_n10|SM_LIB=$GRAFT_REPO_ROOT/variants/u1n10/libstereomst.so|" "e_n13|SM_LIB=$GRAFT_REPO_ROOT/variants/u1n13/libstereomst.so|" || exit 5
