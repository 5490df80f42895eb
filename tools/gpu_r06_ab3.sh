# round 6 A/B 3: 8-wave chain workgroups (variants) on the N = 8 shares and C2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
E="--emulate-rank 0/8 --frame-groups 1"
V1=SM_LIB=variants/cw8/libstereomst.so
V2=SM_LIB=variants/cw8ns8/libstereomst.so
BASE_ARGS="--steps 20 --warmup 5 --no-cpu --no-host-io --no-pms --no-segment" bash tools/gpu_ab.sh \
  "share||$E" "share_cw8|$V1|$E" "share_cw8ns8|$V2|$E" \
  "d||$E --shard d" "d_cw8|$V1|$E --shard d" "d_cw8ns8|$V2|$E --shard d" \
  "c2||" "c2_cw8|$V1|" \
  "share2||$E" "share_cw8_2|$V1|$E" "share_cw8ns8_2|$V2|$E" || exit 3
echo done
