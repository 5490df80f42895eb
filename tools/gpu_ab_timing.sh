# MST/layout parity subset, then bench with and without per-launch HIP events
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mst or tree or full_size_c2_match or match_bitexact_golden or pieces_match" > gpurun_out/tq.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 gpurun_out/tq.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bt_ev$i.log 2>&1 || exit 1
SM_NO_KTIMING=1 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bt_noev$i.log 2>&1 || exit 1
done
bash tools/gpu_trace.sh trt 2
