# chain-wave profile (SM_CHAIN_PROF builds) of each build_variants/prof_* on one C2 match
set -o pipefail
mkdir -p gpurun_out/pv
for d in build_variants/prof*/; do
  [ -d "$d" ] || continue
  n=$(basename $d)
  SM_LIB=$PWD/$d/libstereomst.so timeout -k 10 200 python tools/chain_prof_run.py > gpurun_out/pv/$n.log 2>&1 || { echo "$n FAILED"; exit 1; }
  echo "== $n"; grep -E "len (1[0-9]{4})" gpurun_out/pv/$n.log
done
