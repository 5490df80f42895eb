# round 6 A/B 6: deeper frame pipelines (frames in flight) x HIP hardware queues
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
E="--emulate-rank 0/8 --frame-groups 1"
BASE_ARGS="--steps 40 --warmup 5 --no-cpu --no-host-io --no-pms --no-segment" bash tools/gpu_ab.sh \
  "share||$E" "share_if6||$E --inflight 6" "share_if8||$E --inflight 8" "share_if12||$E --inflight 12" \
  "share_if8_q16|GPU_MAX_HW_QUEUES=16|$E --inflight 8" "share_if12_q16|GPU_MAX_HW_QUEUES=16|$E --inflight 12" \
  "d||$E --shard d" "d_if6||$E --shard d --inflight 6" "d_if8_q16|GPU_MAX_HW_QUEUES=16|$E --shard d --inflight 8" \
  "fg2||--emulate-rank 0/8 --frame-groups 2" "fg2_if6||--emulate-rank 0/8 --frame-groups 2 --inflight 6" \
  "c2||" "c2_if6||--inflight 6" "c2_if6_q16|GPU_MAX_HW_QUEUES=16|--inflight 6" || exit 3
echo done
