set -o pipefail
for D in 64 128 256; do
D=$D SM_LIB=$PWD/build_variants/prof/libstereomst.so timeout -k 10 200 python tools/chain_prof_run.py > gpurun_out/cp_$D.log 2>&1 || exit 1
echo "== D=$D"; grep -E "len (1[0-9]{4})" gpurun_out/cp_$D.log
done
