set -o pipefail
mkdir -p gpurun_out/fill
for r in 1 2; do
for spec in "base:X=1" "f16k:SM_WALK_FILL=16384 SM_WALK_FILL_DN=16384" "f32k:SM_WALK_FILL=32768 SM_WALK_FILL_DN=32768" "f4k:SM_WALK_FILL=4096 SM_WALK_FILL_DN=4096"; do
  name=${spec%%:*}; vars=${spec#*:}
  env $vars timeout -k 10 200 python bench.py --steps 16 --warmup 4 --no-cpu --no-host-io --emulate-rank 0/8 --shard vd > gpurun_out/fill/$name.$r.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/fill/$name.$r.log').read().strip().splitlines()[-1]);print('%-6s %d %.3f' % ('$name', $r, d['ms_per_step']), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
done
done
