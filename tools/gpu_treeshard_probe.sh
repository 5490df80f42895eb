# Does a rank's per-frame floor scale with its tree size?  One view, N=8 view-group slices (64) and
# one view with all 256 slices, on full / half / quarter width images (proxy for subtree shards).
set -o pipefail
O=gpurun_out/tsp
mkdir -p $O
B="python bench.py --steps 12 --warmup 3 --no-cpu --no-host-io --no-pms --disp 256 --height 1200"
for spec in "1920 0/8" "960 0/8" "480 0/8" "960 0/2" "480 0/2"; do
  set -- $spec
  n=w$1_$(echo $2 | tr / _)
  timeout -k 10 200 $B --width $1 --emulate-rank $2 --shard vd > $O/$n.log 2>&1 || exit 2
done
for f in $O/*.log; do
  python3 -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('%-12s %7.3f ms/frame  latency %7.3f  %s %s' % ('$(basename $f .log)', d['ms_per_step'], d['latency_ms_per_frame'], d['config']['workload'], d['kernels_ms_per_step']))"
done
