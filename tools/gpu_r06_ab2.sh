# round 6 A/B 2: chain run sizing (SM_RUN_DIV, dev library) on the N = 8 shares and C2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
E="--emulate-rank 0/8 --frame-groups 1"
DEV=SM_LIB=stereomatch_amd/libstereomst_dev.so
BASE_ARGS="--steps 20 --warmup 5 --no-cpu --no-host-io --no-pms --no-segment" bash tools/gpu_ab.sh \
  "share_dev|$DEV|$E" "share_rd768|$DEV SM_RUN_DIV=768|$E" "share_rd1536|$DEV SM_RUN_DIV=1536|$E" "share_rd192|$DEV SM_RUN_DIV=192|$E" \
  "d_dev|$DEV|$E --shard d" "d_rd768|$DEV SM_RUN_DIV=768|$E --shard d" \
  "c2_dev|$DEV|" "c2_rd256|$DEV SM_RUN_DIV=256|" "c2_rd576|$DEV SM_RUN_DIV=576|" "c2_rd768|$DEV SM_RUN_DIV=768|" \
  "share_dev2|$DEV|$E" "share_rd768_2|$DEV SM_RUN_DIV=768|$E" "c2_dev2|$DEV|" || exit 3
echo done
