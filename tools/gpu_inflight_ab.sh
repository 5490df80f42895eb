# Frames in flight x HIP hardware queues A/B (per-rank N=8 view-group share and C2).
# Usage (on the box): bash tools/gpu_inflight_ab.sh
set -o pipefail
mkdir -p gpurun_out/ifab
run() {  # name, env, bench args
  env $2 timeout -k 10 200 python bench.py --steps 16 --warmup 4 --no-cpu --no-host-io $3 > gpurun_out/ifab/$1.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/ifab/$1.log').read().strip().splitlines()[-1]);print('%-14s %.3f ms/frame lat %.3f' % ('$1', d['ms_per_step'], d['latency_ms_per_frame']))"
}
E="--emulate-rank 0/8 --shard vd"
for q in 4 8 16; do
  for f in 3 4 6; do
    run "vd_q${q}_f${f}" "GPU_MAX_HW_QUEUES=$q" "$E --inflight $f"
  done
done
for q in 4 8; do
  for f in 3 4; do
    run "c2_q${q}_f${f}" "GPU_MAX_HW_QUEUES=$q" "--inflight $f"
  done
done
