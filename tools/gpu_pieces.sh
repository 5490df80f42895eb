# Piece-engine iteration: piece parity tests, full-size C2 parity, bench (+ A/B without pieces),
# repair statistics, kernel trace.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "pieces or full_size_c2 or match_bitexact or aggregate_bitexact" > gpurun_out/tp.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 gpurun_out/tp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/b.log 2>&1
rc=$?; echo "bench exit $rc"; [ $rc -eq 0 ] || exit $rc
SM_NO_PIECES=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/b_nopieces.log 2>&1 || exit 1
SM_PIECE_DEBUG=2 timeout -k 10 120 python bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/pdbg.log 2>&1 || exit 1
bash tools/gpu_trace.sh ${1:-trp} 2
