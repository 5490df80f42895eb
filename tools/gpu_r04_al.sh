# round 4: forest BFS narrow levels -- the next level's loads ahead of the stores -> gpurun_out/r04al
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04al
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_pms_gpu.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 2 > $O/pms100.log 2>&1 || exit 2
python3 - $O/pms100.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["gpu"]
print("frame %.1f ms  prep %.1f (forest %.1f)  first %.1f  later %.1f  spec passes %d serial trees %d" % (d["total_ms"], d["prep_ms"], d.get("prep_forest_ms", 0), d["iter0_ms"], d["iters_ms"], d["spec_rounds"], d["serial_trees"]))
PY
