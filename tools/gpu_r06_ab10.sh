# round 6 A/B 10: where the compact-row build loses C2 time -- one allocation for A + fix rows (variants/onebuf),
# no debug-row store in the walker (variants/noadbg), against the committed build and the product
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ab10
mkdir -p $O
P="--dev --steps 20 --warmup 5 --no-cpu --no-host-io --no-pms --no-segment"
for r in 1 2; do
  for v in head new onebuf noadbg; do
    if [ $v = new ]; then L=""; else L=variants/$v/libstereomst.so; fi
    SM_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace -d $O/${v}_$r -o run -- python bench.py $P > $O/${v}_$r.log 2>&1 || exit 4
  done
done
echo done
