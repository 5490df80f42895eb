# round 4: up chain: results stored by a storer wave
# -> gpurun_out/r04w
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04w
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_pms_gpu.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 2 > $O/pms100_$tag.log 2>&1 || return 1
  python3 - $O/pms100_$tag.log $tag <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["gpu"]
print("%-10s frame %.1f ms  prep %.1f (forest %.1f)  first %.1f %s  later %.1f %s  spec passes %d serial trees %d" % (sys.argv[2], d["total_ms"], d["prep_ms"], d.get("prep_forest_ms", 0), d["iter0_ms"], [round(x, 1) for x in d["first_ms_view"]], d["iters_ms"], [round(x, 1) for x in d["later_ms_view"]], d["spec_rounds"], d["serial_trees"]))
PY
}
run default SM_PMS_X=0 || exit 2


SM_PMS_PROF=1 SM_PMS_SEQ_VIEWS=1 timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 3 --reps 1 > $O/pms3_prof.log 2>&1 || exit 5
grep "pms prof" $O/pms3_prof.log | cut -c1-40,150-
SM_PMS_SEQ_VIEWS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/raw -o run --output-format csv -- python3 tools/pms_bench.py 1920 1200 128 20 --reps 1 > $O/prof.log 2>&1 || exit 6
f=$(find $O/raw -name '*kernel_trace.csv' | head -1); cp "$f" $O/kernel_trace_pms20_seq.csv
f=$(find $O/raw -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_pms20_seq.csv
rm -rf $O/raw
echo traced
