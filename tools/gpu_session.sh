# One GPU session (edited per session; logs under gpurun_out/s/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s
timeout -k 10 900 python -u -m pytest tests/test_pms_gpu.py -x -q --timeout 400 --timeout-method thread > gpurun_out/s/tests_pms.log 2>&1; rc=$?; tail -3 gpurun_out/s/tests_pms.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python tools/pms_bench.py 1920 1200 128 100 --reps 2 > gpurun_out/s/pms100.log 2>&1 || exit 4
tail -1 gpurun_out/s/pms100.log | cut -c1-1200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s/stats1 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu --no-host-io --no-pms --inflight 1 > gpurun_out/s/stats1_bench.log 2>&1 || exit 5
f=$(find gpurun_out/s/stats1 -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/s/kernel_stats_1frame.csv; rm -rf gpurun_out/s/stats1
head -45 gpurun_out/s/kernel_stats_1frame.csv | cut -d, -f1-4 | cut -c1-110
