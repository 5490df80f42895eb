# A/B of runtime knobs (env vars) on the GPU box: each argument is "NAME=VALUE[,NAME=VALUE...]" or
# "base"; each runs a short single-frame bench and prints ms/frame and the per-family times.
# Usage (on the box): bash tools/gpu_ab_env.sh base SM_RUN_DIV=192 "SM_RUN_DIV=128,SM_RUN_CAP=2048"
set -o pipefail
mkdir -p gpurun_out/ab
i=0
for spec in "$@"; do
  i=$((i+1))
  envs=""
  [ "$spec" != "base" ] && envs=$(echo "$spec" | tr ',' ' ')
  env $envs timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-host-io --inflight 1 ${BENCH_ARGS} > gpurun_out/ab/$i.log 2>&1 || exit 5
  python3 -c "import json;d=json.loads(open('gpurun_out/ab/$i.log').read().strip().splitlines()[-1]);print('$spec', round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
done
