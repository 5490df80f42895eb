# round 6 A/B 8: compact A rows -- tile-ordered rows (product) vs rows at the slot (variants/aslot) vs the committed build
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ab8
mkdir -p $O
H=SM_LIB=variants/head/libstereomst.so
S=SM_LIB=variants/aslot/libstereomst.so
REPS=3 bash tools/gpu_ab.sh "head|$H|" "new||" "aslot|$S|" || exit 3
P="--dev --steps 5 --warmup 2 --no-cpu --no-host-io --no-pms --no-segment --inflight 1"
SM_LIB=variants/aslot/libstereomst.so timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_aslot -o run -- python bench.py $P > $O/prof_aslot.log 2>&1 || exit 4
echo done
