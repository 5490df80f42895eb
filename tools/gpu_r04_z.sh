# round 4: segment mode, one frame in flight, kernel trace (where the sweep's 6 ms go) -> gpurun_out/r04z
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04z
mkdir -p $O
SM_SEG_DEBUG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/raw -o run --output-format csv -- python3 bench.py --segment-c 5000 --min-size 200 --inflight 1 --steps 4 --warmup 2 --no-cpu --no-pms > $O/seg1.log 2>&1 || exit 1
f=$(find $O/raw -name '*kernel_trace.csv' | head -1); cp "$f" $O/kernel_trace_seg1.csv
f=$(find $O/raw -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_seg1.csv
rm -rf $O/raw
tail -1 $O/seg1.log | cut -c1-300
