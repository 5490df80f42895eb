# round 6 A/B 5: frames in flight x HIP hardware queues on the N = 8 share and C2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
E="--emulate-rank 0/8 --frame-groups 1"
BASE_ARGS="--steps 30 --warmup 5 --no-cpu --no-host-io --no-pms --no-segment" bash tools/gpu_ab.sh \
  "share||$E" "share_q8|GPU_MAX_HW_QUEUES=8|$E" "share_if4_q8|GPU_MAX_HW_QUEUES=8|$E --inflight 4" \
  "share_if6_q8|GPU_MAX_HW_QUEUES=8|$E --inflight 6" "share_if6_q16|GPU_MAX_HW_QUEUES=16|$E --inflight 6" \
  "share_if4_q16|GPU_MAX_HW_QUEUES=16|$E --inflight 4" \
  "c2||" "c2_q8|GPU_MAX_HW_QUEUES=8|" "c2_if4_q8|GPU_MAX_HW_QUEUES=8|--inflight 4" || exit 3
echo done
