# Diagnostic: build an instrumented copy of the library (-DSM_CHAIN_PROF) into gpurun_out/prof_lib$TAG and
# run one C2 match through it; the chain waves print their cycle / spin counts.
set -o pipefail
mkdir -p gpurun_out/prof_lib$TAG/build
make -s -C stereomatch_amd/csrc OBJ=$GRAFT_REPO_ROOT/gpurun_out/prof_lib$TAG/build OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_lib$TAG/libstereomst.so \
    FLAGS="--offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -std=c++17 -DSM_CHAIN_PROF $EXTRA" -j8 > gpurun_out/prof_build.log 2>&1 || exit 1
SM_LIB=$GRAFT_REPO_ROOT/gpurun_out/prof_lib$TAG/libstereomst.so timeout -k 10 300 python tools/chain_prof_run.py > gpurun_out/chain_prof$TAG.log 2>&1
