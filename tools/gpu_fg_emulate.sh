# Per-rank cost at N = 8 with 2 frame groups (default) and without (bench.py --emulate-rank), plus the
# view-group reduce tests at n = 4 and 8 -> gpurun_out/fg
set -o pipefail
O=gpurun_out/fg
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "view_group_shard_with_reduce" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 12 --warmup 3 --no-cpu --no-host-io --no-pms"
timeout -k 10 200 $B --disp 256 > $O/c4_1gpu.log 2>&1 || exit 1
for spec in "0/8" "2/8" "5/8"; do
  n=$(echo $spec | tr / _)
  timeout -k 10 200 $B --emulate-rank $spec > $O/fg2_$n.log 2>&1 || exit 2
done
timeout -k 10 200 $B --emulate-rank 0/8 --frame-groups 1 > $O/fg1_0_8.log 2>&1 || exit 3
for f in $O/*.log; do
  case $f in *tests.log) continue;; esac
  python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);e=d.get('emulated_rank') or {};print('%-10s %7.3f ms/own frame  stream %s ms/frame  %s' % ('$(basename $f .log)', d['ms_per_step'], round(e.get('stream_ms_per_frame', d['ms_per_step']),3), d['config']['workload']))"
done
