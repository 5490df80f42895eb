# walker iteration: parity subset (odd widths, golden, full C2), bench x2, SQ counters
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "match_bitexact or aggregate or cost_volume or full_size or flir or pieces_match" > gpurun_out/tw.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 gpurun_out/tw.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bw$i.log 2>&1 || exit 1; done
bash tools/gpu_sq.sh sqw
