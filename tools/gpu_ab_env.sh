# A/B of an environment switch on one box: bash tools/gpu_ab_env.sh VAR=value (3 alternations)
set -o pipefail
mkdir -p gpurun_out/abe
for i in $(seq 1 ${ROUNDS:-3}); do
  for m in base alt; do
    if [ $m = alt ]; then env_set="$1"; else env_set="SM_AB_NONE=1"; fi
    env $env_set timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/abe/$m.$i 2>&1 || { echo "$m FAILED"; exit 1; }
    python - gpurun_out/abe/$m.$i $m <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], "ms/frame %.3f" % d['ms_per_step'], {k: round(v,3) for k,v in d['stages_ms'].items() if k in ('mst_ms','layout_ms','up_ms','down_ms')})
PY
  done
done
