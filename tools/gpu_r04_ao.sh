# round 4: segment mode -- global rounds before the LDS tail (env only) -> gpurun_out/r04ao
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ao
mkdir -p $O
lat() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --segment-c 5000 --min-size 200 --steps 8 --warmup 2 --no-cpu --no-pms > $O/lat_$tag.log 2>&1 || return 1
  python3 -c "import json;d=json.loads(open('$O/lat_$tag.log').read().strip().splitlines()[-1]);print('$tag', 'latency %.2f ms' % d['latency_ms_per_frame'], 'stream %.2f ms/frame' % d['ms_per_step'])"
}
lat default SM_SEG_X=0 || exit 1
lat rounds3 SM_SEG_GLOBAL_ROUNDS=3 || exit 2
lat rounds1 SM_SEG_GLOBAL_ROUNDS=1 || exit 3
lat default2 SM_SEG_X=0 || exit 4
lat rounds3b SM_SEG_GLOBAL_ROUNDS=3 || exit 5
