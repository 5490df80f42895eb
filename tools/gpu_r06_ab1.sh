# round 6 A/B 1: parity of the 32-slice half-wave walkers, then share / d-split / C2 timing variants
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ab1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -k "dpad32 or one_view or c4_shard or c4_view_group or subpixel_shard or smoke or degenerate" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 2; }
tail -1 $O/tests.log
E="--emulate-rank 0/8 --frame-groups 1"
BASE_ARGS="--steps 20 --warmup 5 --no-cpu --no-host-io --no-pms --no-segment" bash tools/gpu_ab.sh \
  "d_new||$E --shard d" "d_old|SM_LIB=stereomatch_amd/libstereomst_dev.so SM_NO_HALF_WAVE=1|$E --shard d" \
  "share||$E" "share_lp64|SM_LIB=variants/lp64/libstereomst.so|$E" "share_lp48|SM_LIB=variants/lp48/libstereomst.so|$E" \
  "share_if4||$E --inflight 4" "share_if5||$E --inflight 5" \
  "c2||" "c2_lp64|SM_LIB=variants/lp64/libstereomst.so|" "c2_lp48|SM_LIB=variants/lp48/libstereomst.so|" \
  "d_new2||$E --shard d" "share2||$E" "c2_2||" || exit 3
echo done
