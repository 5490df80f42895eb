# A/B timing of compile-time variants on the GPU box: builds each variant of the library into
# gpurun_out/var_<name>/ and runs a short bench through it (SM_LIB), then the product build.
# Usage (on the box): bash tools/gpu_exp.sh name1 "-DX" name2 "-DY" ...
# EXP_BENCH_ARGS: extra bench.py arguments (e.g. "--emulate-rank 0/8")
set -o pipefail
mkdir -p gpurun_out
while [ $# -ge 2 ]; do
  d=$GRAFT_REPO_ROOT/gpurun_out/var_$1; mkdir -p $d/obj
  make -s -C stereomatch_amd/csrc OBJ=$d/obj OUT=$d/libstereomst.so \
       FLAGS="--offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -std=c++17 $2" -j16 > $d/build.log 2>&1 || exit 1
  SM_LIB=$d/libstereomst.so timeout -k 10 200 python bench.py --dev --steps 10 --warmup 3 --no-cpu --no-host-io $EXP_BENCH_ARGS > $d/bench.log 2>&1 || exit 2
  python3 -c "import json,sys;d=json.loads(open('$d/bench.log').read().strip().splitlines()[-1]);print('$1', round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
  rm -rf $d/obj
  shift 2
done
timeout -k 10 200 python bench.py --dev --steps 10 --warmup 3 --no-cpu --no-host-io $EXP_BENCH_ARGS > gpurun_out/base_bench.log 2>&1 || exit 3
python3 -c "import json;d=json.loads(open('gpurun_out/base_bench.log').read().strip().splitlines()[-1]);print('base', round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
