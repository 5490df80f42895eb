# A/B of variant builds at C3 (3840x2160, D=256): one bench per variant, twice
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
for v in ${VARIANTS:-base}; do
  if [ $v = base ]; then L=""; else L=$GRAFT_REPO_ROOT/build_variants/$v/libstereomst.so; fi
  SM_LIB=$L timeout -k 10 200 python bench.py --width 3840 --height 2160 --disp 256 --steps 4 --warmup 1 --no-cpu > gpurun_out/vc3_${v}_$i.log 2>&1 || exit 1
done
done
