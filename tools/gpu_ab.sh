# Parameterised A/B timing on the GPU box (replaces the one-off gpu_r04_*.sh scripts).
# Each argument is one run, "label|ENV=V ENV2=V2|bench args" (env and args may be empty), run
# in the order given; REPS (default 1) repeats the whole list interleaved.  A variant library is
# selected with SM_LIB=<path> in the env part.  Prints ms/frame and per-family kernel times.
# Usage (on the box): bash tools/gpu_ab.sh "base||" "fo|SM_EXP_FILTER_ONLY=1|" "if4||--inflight 4"
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab
mkdir -p $O
REPS=${REPS:-1}
BASE_ARGS=${BASE_ARGS:---steps 20 --warmup 5 --no-cpu --no-host-io --no-pms --no-segment}
for rep in $(seq 1 $REPS); do
  for spec in "$@"; do
    label=${spec%%|*}; rest=${spec#*|}; envs=${rest%%|*}; args=${rest#*|}
    log=$O/${label}_$rep.log
    env $envs timeout -k 10 300 python bench.py --dev $BASE_ARGS $args > $log 2>&1 || { echo "FAILED $label"; tail -5 $log; exit 2; }
    python3 - "$label" "$log" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = {a: round(b, 3) for a, b in d["kernels_ms_per_step"].items()}
tf = d["roofline"].get("tree_filter", {})
print("%-14s %.3f ms/frame  lat %.2f  filter wall %.3f  %s" % (sys.argv[1], d["ms_per_step"], d["latency_ms_per_frame"],
      tf.get("wall_ms_per_step", 0), k), flush=True)
EOF
  done
done
