# Build variant copies of libstereomst.so (extra -D flags) under build_variants/<name>/ for A/B runs
# with SM_LIB.  Usage: bash tools/build_variants.sh name1 "-DX=1" name2 "-DY=2" ...
set -e
ROOT=$(cd $(dirname $0)/.. && pwd)
while [ $# -ge 2 ]; do
  d=$ROOT/build_variants/$1; mkdir -p $d/obj
  make -s -C $ROOT/stereomatch_amd/csrc OBJ=$d/obj OUT=$d/libstereomst.so \
       FLAGS="--offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -std=c++17 $2" -j8
  shift 2
done
