# round 4: no run-time-indexed local arrays (PMS chain loaders, forest BFS, SPL = 4 WTA, k_meta)
# -> gpurun_out/r04x
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04x
mkdir -p $O
timeout -k 10 840 python3 -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread \
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
run default SM_PMS_X=0 || exit 2
SM_PMS_PROF=1 SM_PMS_SEQ_VIEWS=1 timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 3 --reps 1 > $O/pms3_prof.log 2>&1 || exit 5
grep "pms prof" $O/pms3_prof.log | cut -c1-40,150-
timeout -k 10 400 python3 bench.py --no-cpu > $O/bench_default.log 2>&1 || exit 6
python3 -c "import json;d=json.loads(open('$O/bench_default.log').read().strip().splitlines()[-1]);print('bench', d['config']['workload'], round(d['ms_per_step'],3), '%.4g' % d['value'], round(d['roofline']['frac'],3))"
timeout -k 10 300 python3 bench.py --no-cpu --no-pms --disp 256 > $O/bench_d256.log 2>&1 || exit 7
python3 -c "import json;d=json.loads(open('$O/bench_d256.log').read().strip().splitlines()[-1]);print('bench d256', d['config']['workload'], round(d['ms_per_step'],3), '%.4g' % d['value'], round(d['roofline']['frac'],3))"
