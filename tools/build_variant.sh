# A variant build of the library for timing A/Bs (never the product): variants/<name>/libstereomst.so
# built with extra compiler flags, e.g.  bash tools/build_variant.sh lp64 -DSM_LONG_PATH=64
# Use it with SM_LIB=variants/<name>/libstereomst.so python bench.py --dev ...
set -e
NAME=$1; shift
D=$(cd "$(dirname "$0")/.." && pwd)/variants/$NAME
mkdir -p $D
make -s -C "$(dirname "$0")/../stereomatch_amd/csrc" -j8 OBJ=$D/obj OUT=$D/libstereomst.so EXTRA="$*" $D/libstereomst.so
echo built $D/libstereomst.so
