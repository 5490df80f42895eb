# round 4: PMS chain threshold 64 by default -- full GPU suite and the 100-call frame -> gpurun_out/r04aq
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04aq
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 2 > $O/pms100_$tag.log 2>&1 || return 1
  python3 - $O/pms100_$tag.log $tag <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["gpu"]
print("%-8s frame %.1f ms  prep %.1f  first %.1f  later %.1f" % (sys.argv[2], d["total_ms"], d["prep_ms"], d["iter0_ms"], d["iters_ms"]))
PY
}
run default SM_PMS_X=0 || exit 3
run cm96 SM_PMS_CHAIN_MIN=96 || exit 4


run cm48 SM_PMS_CHAIN_MIN=48 || exit 7
run default2 SM_PMS_X=0 || exit 8
