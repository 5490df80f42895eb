# Sweep the tile-phase iteration cap (SM_MST_LOCAL_ITERS): MST stage time and tile-kernel time.
set -o pipefail
mkdir -p gpurun_out/sweep
for it in ${ITERS:-1 2 3 4 6 8 64}; do
  SM_MST_LOCAL_ITERS=$it timeout -k 10 200 python bench.py --dev --steps 20 --warmup 3 --no-cpu > gpurun_out/sweep/i$it 2>&1 || { echo "i$it FAILED"; exit 1; }
  echo "iters $it $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sweep/i$it | head -1) $(grep -o '"mst_ms": [0-9.]*' gpurun_out/sweep/i$it)"
done
