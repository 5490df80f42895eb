# One GPU session (edited per session; logs under gpurun_out/s/)
# This session: the final build's other lines: the C3-size batch pair and the guided-filter aggregator at C2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s
timeout -k 10 300 python bench.py --mode batch --steps 6 --warmup 2 --no-cpu > gpurun_out/s/bench_batch.log 2>&1 || exit 4
tail -1 gpurun_out/s/bench_batch.log | cut -c1-200
timeout -k 10 300 python bench.py --aggregator guided --steps 10 --warmup 2 --no-cpu --no-pms --no-segment > gpurun_out/s/bench_guided.log 2>&1 || exit 5
tail -1 gpurun_out/s/bench_guided.log | cut -c1-200
