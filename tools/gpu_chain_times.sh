# Chain-engine occupancy per launch (diagnostic build -DSM_CHAIN_TIMES, one C2 match): see tools/chain_times.py
set -o pipefail
mkdir -p gpurun_out/ct_lib/build
make -s -C stereomatch_amd/csrc OBJ=$GRAFT_REPO_ROOT/gpurun_out/ct_lib/build OUT=$GRAFT_REPO_ROOT/gpurun_out/ct_lib/libstereomst.so \
    FLAGS="--offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -std=c++17 -DSM_CHAIN_TIMES" -j16 > gpurun_out/ct_build.log 2>&1 || exit 1
SM_LIB=$GRAFT_REPO_ROOT/gpurun_out/ct_lib/libstereomst.so timeout -k 10 300 python tools/chain_prof_run.py > gpurun_out/chain_times.log 2>&1 || exit 2
rm -rf gpurun_out/ct_lib/build
python tools/chain_times.py gpurun_out/chain_times.log
