# One GPU session (edited per session; logs under gpurun_out/s/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "mst_ or timeout or layout or match_bitexact_golden or full_size_c2_match or pieces_match or full_size_c3_match or segment" -x -v --timeout 300 --timeout-method thread > gpurun_out/s/tests.log 2>&1; rc=$?; tail -3 gpurun_out/s/tests.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python -u -m pytest tests/test_pms_gpu.py -k "cycle or golden_bitexact or forest_matches" -x -q --timeout 200 --timeout-method thread > gpurun_out/s/tests_pms.log 2>&1; rc=$?; tail -2 gpurun_out/s/tests_pms.log; [ $rc -eq 0 ] || exit 7
REPS=2 bash tools/gpu_ab.sh "prev|SM_LIB=$GRAFT_REPO_ROOT/variants/prev/libstereomst.so|" "new||" "skl|SM_EXP_SKIP=layout|" || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s/stats1 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu --no-host-io --no-pms --no-segment --inflight 1 > gpurun_out/s/stats1_bench.log 2>&1 || exit 5
f=$(find gpurun_out/s/stats1 -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/s/kernel_stats_1frame.csv; rm -rf gpurun_out/s/stats1
