# Run tools/chain_prof_run.py through each build_variants/*/libstereomst.so (SM_CHAIN_PROF builds)
set -o pipefail
mkdir -p gpurun_out/cv
for d in build_variants/*/; do
  n=$(basename $d)
  SM_LIB=$PWD/$d/libstereomst.so timeout -k 10 200 python tools/chain_prof_run.py > gpurun_out/cv/$n.log 2>&1 || { echo "$n FAILED"; exit 1; }
  echo "== $n"; grep -E "len (1[0-9]{4})" gpurun_out/cv/$n.log
done
