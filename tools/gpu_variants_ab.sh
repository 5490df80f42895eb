# A/B of variant builds (build_variants/<name>/libstereomst.so via SM_LIB): parity subset + bench
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-base w8a w8b w8c w16r}; do
  if [ $v = base ]; then L=""; else L=$GRAFT_REPO_ROOT/build_variants/$v/libstereomst.so; fi
  SM_LIB=$L timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pieces_match or full_size_c2_match" > gpurun_out/va_$v.log 2>&1
  rc=$?; echo "$v tests $rc"; [ $rc -eq 0 ] || exit $rc
  for i in 1 2; do SM_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/vb_${v}_$i.log 2>&1 || exit 1; done
done
