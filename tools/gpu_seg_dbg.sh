# segment_gpu phase timings (SM_SEG_DEBUG) over a few segment-mode frames
set -o pipefail
mkdir -p gpurun_out/segdbg
SM_SEG_DEBUG=1 timeout -k 10 300 python bench.py --dev --segment-c 5000 --no-cpu --no-pms --steps 4 --warmup 1 --inflight 1 > gpurun_out/segdbg/bench.log 2>gpurun_out/segdbg/err.log || exit 1
grep segment_gpu gpurun_out/segdbg/err.log | tail -4
python3 -c "import json;d=json.loads(open('gpurun_out/segdbg/bench.log').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],3), d['stages_ms']['mst_ms'])"
