# round 4: GPU schedule forest after the contention fixes and the LDS frontier -- the forest check, the
# 100-call C2 frame, forest kernel stats of a 2-call run -> gpurun_out/r04p
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04p
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_pms_gpu.py \
  -k "gpu_forest_matches or full_c2_speculative" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 2 > $O/pms100.log 2>&1 || exit 2
python3 - $O/pms100.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["gpu"]
print("frame %.1f ms  prep %.1f (seg %.1f forest %.1f)  first %.1f  later %.1f" % (d["total_ms"], d["prep_ms"], d["prep_seg_ms"], d["prep_forest_ms"], d["iter0_ms"], d["iters_ms"]))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/raw -o run --output-format csv -- python3 tools/pms_bench.py 1920 1200 128 2 --reps 1 > $O/prof.log 2>&1 || exit 3
f=$(find $O/raw -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_pms2.csv
f=$(find $O/raw -name '*kernel_trace.csv' | head -1); cp "$f" $O/kernel_trace_pms2.csv
rm -rf $O/raw
grep k_pf_ $O/kernel_stats_pms2.csv | cut -d, -f1-4 | head -12
SM_PMS_PROF=1 SM_PMS_SEQ_VIEWS=1 timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 3 --reps 1 > $O/pms3_prof.log 2>&1 || exit 4
grep "pms prof" $O/pms3_prof.log
