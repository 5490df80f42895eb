# Full GPU suite, then the guided aggregator: bench at C2 and kernel-trace stats.
# Outputs under gpurun_out/guided/.  Usage: bash tools/gpu_guided_round.sh [skip-tests]
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/guided
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
if [ "$1" != "skip-tests" ]; then
  timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 11
fi
timeout -k 10 300 python bench.py --aggregator guided --no-cpu --steps 10 --warmup 2 > $O/bench_guided.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python bench.py --aggregator guided --steps 5 --warmup 1 --no-cpu --no-host-io --inflight 1 > $O/stats_bench.log 2>&1 || exit 13
echo done
