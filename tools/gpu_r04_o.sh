# round 4: PMS chain knobs (ring depth, threshold), 100-call C2 frame per setting, and a 20-call kernel trace
# with the views one after the other -> gpurun_out/r04o
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04o
mkdir -p $O
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 2 > $O/pms100_$tag.log 2>&1 || return 1
  python3 - $O/pms100_$tag.log $tag <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["gpu"]
print("%-14s frame %.1f ms  prep %.1f (forest %.1f)  first %.1f  later %.1f  views first %s later %s" % (sys.argv[2], d["total_ms"], d["prep_ms"], d.get("prep_forest_ms", 0), d["iter0_ms"], d["iters_ms"], [round(x, 1) for x in d["first_ms_view"]], [round(x, 1) for x in d["later_ms_view"]]))
PY
}
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_pms_gpu.py \
  -k "gpu_forest_matches or synthetic_modes or full_c2_speculative" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "segment" > $O/tests_seg.log 2>&1 || { tail -40 $O/tests_seg.log; exit 1; }
tail -2 $O/tests_seg.log
for e in SM_SEG_X=0 SM_SEG_NOLDS=1; do
  env $e SM_SEG_DEBUG=1 timeout -k 10 300 python bench.py --segment-c 5000 --no-cpu --no-pms --steps 16 --warmup 4 > $O/seg_$e.log 2> $O/seg_$e.err || exit 9
  grep segment_gpu $O/seg_$e.err | tail -1 | cut -c1-200
  python3 -c "import json;d=json.loads(open('$O/seg_$e.log').read().strip().splitlines()[-1]);print('seg $e', round(d['ms_per_step'],3), 'ms/frame, latency', round(d.get('latency_ms_per_frame'),2))"
done
run default SM_PMS_X=0 || exit 2
run nsu2 SM_PMS_CHAIN_NSU=2 || exit 3
run nsu2_nsd7 SM_PMS_CHAIN_NSU=2 SM_PMS_CHAIN_NSD=7 || exit 4
run nsu3 SM_PMS_CHAIN_NSU=3 || exit 5
run cm128 SM_PMS_CHAIN_MIN=128 || exit 6
run cm48 SM_PMS_CHAIN_MIN=48 || exit 6
run cm192 SM_PMS_CHAIN_MIN=192 || exit 6
run piece256 SM_PMS_PIECE=256 || exit 6
run piece384 SM_PMS_PIECE=384 || exit 6
SM_PMS_PROF=1 SM_PMS_SEQ_VIEWS=1 timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 2 --reps 1 > $O/pms2_prof.log 2>&1 || exit 8
grep "pms prof" $O/pms2_prof.log
SM_PMS_SEQ_VIEWS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/raw -o run --output-format csv -- python3 tools/pms_bench.py 1920 1200 128 20 --reps 1 > $O/prof.log 2>&1 || exit 7
f=$(find $O/raw -name '*kernel_trace.csv' | head -1); cp "$f" $O/kernel_trace_pms20_seq.csv
f=$(find $O/raw -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_pms20_seq.csv
rm -rf $O/raw
echo traced
