# GPU round trip: parity tests (optionally filtered), then a short bench; stops at the first failure.
# Usage: bash tools/gpu_check.sh "<pytest -k expr>" <bench steps>
set -o pipefail
mkdir -p gpurun_out
K="${1:-not full_size and not flir_c1}"
STEPS="${2:-5}"
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "$K" > gpurun_out/t.log 2>&1
rc=$?; echo "tests exit $rc" | tee -a gpurun_out/t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps $STEPS --warmup 2 --no-cpu > gpurun_out/b.log 2>&1
rc=$?; echo "bench exit $rc"
exit $rc
