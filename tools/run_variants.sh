# On the GPU box: bench each build_variants/*/libstereomst.so (quick parity subset first).
set -o pipefail
mkdir -p gpurun_out/variants
for d in build_variants/*/; do
  n=$(basename $d)
  SM_LIB=$PWD/$d/libstereomst.so timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "match_synthetic or full_size_c2_match" > gpurun_out/variants/$n.t 2>&1 || { echo "$n tests FAILED"; continue; }
  SM_LIB=$PWD/$d/libstereomst.so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/variants/$n.b 2>&1 || { echo "$n bench FAILED"; exit 1; }
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/variants/$n.b) $(grep -o '"kernels_ms_per_step": {[^}]*}' gpurun_out/variants/$n.b)"
done
