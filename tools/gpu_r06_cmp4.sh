# round 6: compact A rows, final form -- layout invariants, smoke + suite, C3 with 2 vs 3 frames in flight
set -o pipefail
TAG=${1:-r06cmp4}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/layout_check.py > $O/layout_check.log 2>&1 || { cat $O/layout_check.log; exit 1; }
bash tools/gpu_tests.sh $TAG || exit 2
B="--mode batch --steps 10 --warmup 3 --no-cpu --no-host-io --no-pms --no-segment"
for r in 1 2; do
  timeout -k 10 400 python bench.py $B --inflight 2 > $O/c3_if2_$r.log 2>&1 || exit 3
  timeout -k 10 400 python bench.py $B > $O/c3_$r.log 2>&1 || exit 4
done
for f in $O/c3_*.log; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f'.split('/')[-1], round(d['ms_per_step'],3), 'inflight', d['frames_in_flight'])"; done
echo done
