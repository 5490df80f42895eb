# round 4: segment mode -- LDS tails over the still-crossing edges, hashed pair dedupe
# onesweep sorts -> gpurun_out/r04ar
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ar
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "seg" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
lat() {  # tag, env...: segment-mode single-frame latency and streamed ms/frame
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --segment-c 5000 --min-size 200 --steps 8 --warmup 2 --no-cpu --no-pms > $O/lat_$tag.log 2>&1 || return 1
  python3 -c "import json;d=json.loads(open('$O/lat_$tag.log').read().strip().splitlines()[-1]);print('$tag', 'latency %.2f ms' % d['latency_ms_per_frame'], 'stream %.2f ms/frame' % d['ms_per_step'])"
}
lat default SM_SEG_X=0 || exit 2

lat tailglobal SM_SEG_TAIL_GLOBAL=1 || exit 7

lat default2 SM_SEG_X=0 || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/raw -o run --output-format csv -- python3 bench.py --segment-c 5000 --min-size 200 --inflight 1 --steps 4 --warmup 2 --no-cpu --no-pms > $O/seg1.log 2>&1 || exit 5
f=$(find $O/raw -name '*kernel_trace.csv' | head -1); cp "$f" $O/kernel_trace_seg1.csv
rm -rf $O/raw
echo traced
SM_SEG_PROF=1 timeout -k 10 300 python3 bench.py --segment-c 5000 --min-size 200 --inflight 1 --steps 2 --warmup 1 --no-cpu --no-pms > $O/prof.log 2>&1 || exit 6
grep "seg prof" $O/prof.log | tail -2 | cut -c1-300
