# Per-rank cost of the strong-mode partitions on one GPU (bench.py --emulate-rank, no collective),
# plus the unsharded C4-size frame: inputs of the multi-GPU estimate in DESIGN.md 7.
# Usage (on the box): bash tools/gpu_emulate.sh  -> gpurun_out/emu/*.log
set -o pipefail
O=gpurun_out/emu
mkdir -p $O
B="python bench.py --steps 12 --warmup 3 --no-cpu --no-host-io --no-pms"
timeout -k 10 200 $B --disp 256 > $O/c4_1gpu.log 2>&1 || exit 1
for spec in "0/8 vd" "0/8 d" "4/8 vd" "0/4 vd" "0/2 vd" "0/2 d"; do
  set -- $spec
  n=$(echo $1 | tr / _)_$2
  timeout -k 10 200 $B --emulate-rank $1 --shard $2 > $O/$n.log 2>&1 || exit 2
done
for f in $O/*.log; do
  python3 -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('%-16s %7.3f ms/frame  latency %7.3f  %s' % ('$(basename $f .log)', d['ms_per_step'], d['latency_ms_per_frame'], d['stages_ms']))"
done
