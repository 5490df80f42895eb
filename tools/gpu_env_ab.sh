# Interleaved A/B of runtime environment knobs on the GPU box (same library, short benches).
# Usage: bash tools/gpu_env_ab.sh <repeats> "name1:VAR=x VAR2=y" "name2:VAR=z" ...
set -o pipefail
mkdir -p gpurun_out/envab
R=$1; shift
for r in $(seq 1 $R); do
  for spec in "$@"; do
    name=${spec%%:*}; vars=${spec#*:}
    env $vars timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --no-host-io > gpurun_out/envab/$name.$r.log 2>&1 || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/envab/$name.$r.log').read().strip().splitlines()[-1]);print('%-10s %d %.3f wall %.3f' % ('$name', $r, d['ms_per_step'], d['roofline']['tree_filter']['wall_ms_per_step']), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
  done
done
