# segment GPU tests, phase timings, pipelined segment-mode bench lines
set -o pipefail
bash tools/gpu_seg_dbg.sh || exit 1
mkdir -p gpurun_out/seg
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "segment or pms" --timeout 300 --timeout-method thread > gpurun_out/seg/tests.log 2>&1
rc=$?; tail -3 gpurun_out/seg/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_seg_bench.sh
