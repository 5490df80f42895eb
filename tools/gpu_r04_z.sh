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
lat() {  # tag, env...: segment-mode single-frame latency and streamed ms/frame
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --segment-c 5000 --min-size 200 --steps 8 --warmup 2 --no-cpu --no-pms > $O/lat_$tag.log 2>&1 || return 1
  python3 -c "import json;d=json.loads(open('$O/lat_$tag.log').read().strip().splitlines()[-1]);print('$tag', 'latency %.2f ms' % d['latency_ms_per_frame'], 'stream %.2f ms/frame' % d['ms_per_step'])"
}
lat default SM_SEG_X=0 || exit 2
lat rounds1 SM_SEG_GLOBAL_ROUNDS=1 || exit 3
lat rounds3 SM_SEG_GLOBAL_ROUNDS=3 || exit 4
lat flatten3 SM_SEG_FLATTEN=3 || exit 5
lat default2 SM_SEG_X=0 || exit 6
