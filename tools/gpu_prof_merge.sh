set -o pipefail
mkdir -p gpurun_out/pm
SM_LIB=$PWD/build_variants/prof_merge/libstereomst.so timeout -k 10 200 python tools/chain_prof_run.py > gpurun_out/pm/merge.log 2>&1 || exit 1
SM_NO_MERGE=1 SM_LIB=$PWD/build_variants/prof_merge/libstereomst.so timeout -k 10 200 python tools/chain_prof_run.py > gpurun_out/pm/nomerge.log 2>&1 || exit 1
echo "== merge"; grep -E "len (1[0-9]{4})" gpurun_out/pm/merge.log
echo "== nomerge"; grep -E "len (1[0-9]{4})" gpurun_out/pm/nomerge.log
