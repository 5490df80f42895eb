# One GPU session (edited per session; logs under gpurun_out/s/)
# This session: the up chain's next-half reads pinned ahead of the recurrence by a scheduling barrier
# (-DSM_UP_SB), with two or three register sets (-DSM_UP_PIPE3): chain-wave cycles (prof builds), the GPU
# parity suite through the SB builds, an interleaved C2 A/B and the N = 8 share against the in-tree build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s
V=$GRAFT_REPO_ROOT/variants
for v in prof sbp p3sbp; do
  SM_LIB=$V/$v/libstereomst.so timeout -k 10 300 python tools/chain_prof_run.py > gpurun_out/s/cp_$v.log 2>&1 || exit 2
  echo "== $v"; grep -E "^up chain" gpurun_out/s/cp_$v.log | sort -t' ' -k6 -n -r | head -3 || true
done
for v in sb p3sb; do
  SM_LIB=$V/$v/libstereomst.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/s/tests_$v.log 2>&1; rc=$?; tail -1 gpurun_out/s/tests_$v.log; [ $rc -eq 0 ] || exit 7
done
REPS=2 bash tools/gpu_ab.sh "base||" "sb|SM_LIB=$V/sb/libstereomst.so|" "p3sb|SM_LIB=$V/p3sb/libstereomst.so|" || exit 3
REPS=1 bash tools/gpu_ab.sh "e8base||--emulate-rank 0/8 --frame-groups 1" "e8sb|SM_LIB=$V/sb/libstereomst.so|--emulate-rank 0/8 --frame-groups 1" "e8p3sb|SM_LIB=$V/p3sb/libstereomst.so|--emulate-rank 0/8 --frame-groups 1" || exit 4
