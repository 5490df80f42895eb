# round 6: deterministic compact A rows -- layout invariants first (no filter runs), then smoke + suite,
# context memory, and C2 A/B against the committed build (variants/head)
set -o pipefail
TAG=${1:-r06cmp3}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/layout_check.py > $O/layout_check.log 2>&1 || { cat $O/layout_check.log; exit 1; }
cat $O/layout_check.log
bash tools/gpu_tests.sh $TAG || exit 2
timeout -k 10 300 python tools/mem_probe.py 3840 2160 256 > $O/mem_c3.log 2>&1 || exit 4
timeout -k 10 300 python tools/mem_probe.py 1920 1200 128 > $O/mem_c2.log 2>&1 || exit 5
cat $O/mem_c3.log $O/mem_c2.log | grep context
H=SM_LIB=variants/head/libstereomst.so
REPS=3 bash tools/gpu_ab.sh "head|$H|" "new||" || exit 6
P="--dev --steps 5 --warmup 2 --no-cpu --no-host-io --no-pms --no-segment --inflight 1"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_new -o run -- python bench.py $P > $O/prof_new.log 2>&1 || exit 7
echo done
