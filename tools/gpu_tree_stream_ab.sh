# Tree stages on a low-priority stream (default) vs one stream per context (SM_TREE_STREAM=0):
# parity suite, then interleaved A/B of C2 and the N=8 view-group share.
set -o pipefail
mkdir -p gpurun_out/ts
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/t_ts.log 2>&1
rc=$?; echo "tests exit $rc" >> gpurun_out/t_ts.log; tail -3 gpurun_out/t_ts.log
[ $rc -eq 0 ] || exit $rc
run() {
  env $2 timeout -k 10 200 python bench.py --steps 16 --warmup 4 --no-cpu --no-host-io $3 > gpurun_out/ts/$1.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/ts/$1.log').read().strip().splitlines()[-1]);r=d['roofline'];print('%-10s %.3f ms/frame lat %.3f frac %.3f' % ('$1', d['ms_per_step'], d['latency_ms_per_frame'], r['frac']))"
}
for r in 1 2; do
  run c2_one "SM_TREE_STREAM=0" ""
  run c2_ts "SM_TREE_STREAM=1" ""
  run c2_ts_q8 "SM_TREE_STREAM=1 GPU_MAX_HW_QUEUES=8" ""
  run vd8_one "SM_TREE_STREAM=0" "--emulate-rank 0/8 --shard vd"
  run vd8_ts "SM_TREE_STREAM=1" "--emulate-rank 0/8 --shard vd"
  run vd8_ts_q8 "SM_TREE_STREAM=1 GPU_MAX_HW_QUEUES=8" "--emulate-rank 0/8 --shard vd"
done
