# Final-build bench lines of the other modes: segment (c=5000, its default 6 in flight), guided, and
# the N=8 frame-group rank emulation -> gpurun_out/modes
set -o pipefail
O=gpurun_out/modes
mkdir -p $O
timeout -k 10 300 python bench.py --segment-c 5000 --no-cpu --no-pms --steps 16 --warmup 4 > $O/segment.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --aggregator guided --no-cpu --no-pms --steps 10 --warmup 2 > $O/guided.log 2>&1 || exit 2
timeout -k 10 200 python bench.py --steps 12 --warmup 3 --no-cpu --no-host-io --no-pms --emulate-rank 0/8 > $O/emu_0_8.log 2>&1 || exit 3
for f in segment guided emu_0_8; do
  python3 -c "import json;d=json.loads(open('$O/$f.log').read().strip().splitlines()[-1]);e=d.get('emulated_rank') or {};print('$f', round(d['ms_per_step'],3), e.get('stream_ms_per_frame'), d['config']['workload'])"
done
