# Segment-mode bench lines (C2, c=5000, min_size=200) at 3 / 6 / 8 frames in flight
set -o pipefail
O=gpurun_out/segb
mkdir -p $O
for n in ${INFL:-0 4 8}; do
  timeout -k 10 300 python bench.py --segment-c 5000 --no-cpu --no-pms --steps 16 --warmup 4 --inflight $n > $O/seg_$n.log 2>&1 || exit 3
  python3 -c "import json;d=json.loads(open('$O/seg_$n.log').read().strip().splitlines()[-1]);print('inflight $n', round(d['ms_per_step'],3), 'ms/frame; single-frame stages', {k: round(v,2) for k,v in d['stages_ms'].items()})"
done
