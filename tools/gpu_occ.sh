# walker occupancy sweep: SM_WALK_LDS_PAD limits blocks per CU (0 = register-limited default)
set -o pipefail
mkdir -p gpurun_out/occ
for pad in 0 24700 38000 64000 0; do
  SM_WALK_LDS_PAD=$pad timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/occ/p$pad.log 2>&1 || exit 1
  python - gpurun_out/occ/p$pad.log $pad <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
k=d['kernels_ms_per_step']
print("pad", sys.argv[2], "ms %.3f" % d['ms_per_step'], "up_walk %.3f down_walk %.3f" % (k['k_up_walk'], k['k_down_walk']))
PY
done
