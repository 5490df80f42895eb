# round 4: PMS up-chain ring depth re-swept after the scratch fix (env only) -> gpurun_out/r04an
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04an
mkdir -p $O
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 2 > $O/pms100_$tag.log 2>&1 || return 1
  python3 - $O/pms100_$tag.log $tag <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["gpu"]
print("%-8s frame %.1f ms  prep %.1f  first %.1f  later %.1f" % (sys.argv[2], d["total_ms"], d["prep_ms"], d["iter0_ms"], d["iters_ms"]))
PY
}
run default SM_PMS_X=0 || exit 1
run nsu3 SM_PMS_CHAIN_NSU=3 || exit 2
run nsu6 SM_PMS_CHAIN_NSU=6 || exit 3
run nsu8 SM_PMS_CHAIN_NSU=8 || exit 4
run cm64 SM_PMS_CHAIN_MIN=64 || exit 5
run default2 SM_PMS_X=0 || exit 6
