# Quick GPU iteration: parity subset (incl. full-size C2 match), bench, per-launch kernel trace,
# chain-wave profile.  Stops at the first failure.  Usage: bash tools/gpu_quick.sh <trace tag>
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q -k "match_synthetic or aggregate or full_size_c2_match or lr_check or golden" > gpurun_out/t0.log 2>&1
rc=$?; echo "tests exit $rc"; tail -1 gpurun_out/t0.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/b.log 2>&1
rc=$?; echo "bench exit $rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_trace.sh ${1:-trace} 1 || exit 1
[ -n "$NOPROF" ] || bash tools/chain_prof.sh
