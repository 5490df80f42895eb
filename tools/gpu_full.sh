# GPU round trip: quick parity subset first (catches hangs early), then the full GPU suite, bench
# and a kernel trace; stops at the first failure.  Usage: bash tools/gpu_full.sh <trace dir>
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -m pytest tests -m gpu -x -q -k "match_synthetic or aggregate" > gpurun_out/t0.log 2>&1
rc=$?; echo "quick tests exit $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1
rc=$?; echo "tests exit $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/b.log 2>&1
rc=$?; echo "bench exit $rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_trace.sh ${1:-trace} 1
