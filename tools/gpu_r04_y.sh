# round 4: serial PMS kernel thread count (768 default vs 1024 / 512) -> gpurun_out/r04y
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04y
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_pms_gpu.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 2 > $O/pms100_$tag.log 2>&1 || return 1
  python3 - $O/pms100_$tag.log $tag <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["gpu"]
print("%-10s frame %.1f ms  prep %.1f (forest %.1f)  first %.1f %s  later %.1f %s  spec passes %d serial trees %d" % (sys.argv[2], d["total_ms"], d["prep_ms"], d.get("prep_forest_ms", 0), d["iter0_ms"], [round(x, 1) for x in d["first_ms_view"]], d["iters_ms"], [round(x, 1) for x in d["later_ms_view"]], d["spec_rounds"], d["serial_trees"]))
PY
}
run nt768 SM_PMS_SER_NT=768 || exit 2
run nt1024 SM_PMS_SER_NT=1024 || exit 3
run nt512 SM_PMS_SER_NT=512 || exit 4
run nt768b SM_PMS_SER_NT=768 || exit 5
