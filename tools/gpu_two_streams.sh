set -o pipefail
mkdir -p gpurun_out/ts
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --no-host-io > gpurun_out/ts/one.log 2>&1 || exit 1
SM_TWO_STREAMS=1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --no-host-io > gpurun_out/ts/two.log 2>&1 || exit 2
SM_TWO_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ts/tr -o run --output-format csv -- python bench.py --steps 4 --warmup 2 --no-cpu --no-host-io --inflight 1 > gpurun_out/ts/tr.log 2>&1 || exit 3
python tools/trace_frame.py gpurun_out/ts/tr/run_kernel_trace.csv > gpurun_out/ts/timeline_two.txt
for f in one two; do python3 -c "import json;d=json.loads(open('gpurun_out/ts/$f.log').read().strip().splitlines()[-1]);t=d['roofline']['tree_filter'];print('$f', round(d['ms_per_step'],3), 'wall', round(t['wall_ms_per_step'],3), 'sum', round(t['ms_per_step'],3), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})"; done
