# Split calls (sm_match_begin/finish) vs sm_match_async: parity suite, then interleaved A/B of
# the default C2 bench and the per-rank N=8 / N=4 view-group shares.
# Usage (on the box): bash tools/gpu_split_ab.sh
set -o pipefail
mkdir -p gpurun_out/split
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/t_split.log 2>&1
rc=$?; echo "tests exit $rc" >> gpurun_out/t_split.log; tail -3 gpurun_out/t_split.log
[ $rc -eq 0 ] || exit $rc
run() {
  timeout -k 10 200 python bench.py --steps 16 --warmup 4 --no-cpu --no-host-io $2 > gpurun_out/split/$1.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/split/$1.log').read().strip().splitlines()[-1]);print('%-12s %.3f ms/frame lat %.3f' % ('$1', d['ms_per_step'], d['latency_ms_per_frame']), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
}
for r in 1 2; do
  run c2_async "--no-split"
  run c2_split ""
  run vd8_async "--emulate-rank 0/8 --shard vd --no-split"
  run vd8_split "--emulate-rank 0/8 --shard vd"
done
run vd4_split "--emulate-rank 0/4 --shard vd"
run c4_split "--disp 256"
run vd8r_split "--emulate-rank 4/8 --shard vd"
