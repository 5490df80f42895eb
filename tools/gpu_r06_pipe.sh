# Frames in flight and the host pipeline's lag (bench.py --inflight / --lag), C2 and the N = 8 G = 1 share
set -o pipefail
REPS=2 bash tools/gpu_ab.sh "c2_i3l1||" "c2_i4l2||--inflight 4 --lag 2" "c2_i4l1||--inflight 4" "c2_i5l3||--inflight 5 --lag 3" \
  "s8_i3l1||--emulate-rank 0/8 --frame-groups 1" "s8_i4l2||--emulate-rank 0/8 --frame-groups 1 --inflight 4 --lag 2" \
  "s8_i6l4||--emulate-rank 0/8 --frame-groups 1 --inflight 6 --lag 4"
