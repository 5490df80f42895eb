# A/B on one box: alternate bench runs of each build_variants/*/libstereomst.so (ROUNDS times).
set -o pipefail
mkdir -p gpurun_out/ab
for i in $(seq 1 ${ROUNDS:-3}); do
  for d in build_variants/*/; do
    n=$(basename $d)
    SM_LIB=$PWD/$d/libstereomst.so timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/ab/$n.$i 2>&1 || { echo "$n FAILED"; exit 1; }
    echo "$n $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/$n.$i)"
  done
done
