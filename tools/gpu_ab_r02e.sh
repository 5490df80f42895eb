# Round-2 end A/B experiments on the GPU box (each: interleaved short benches, one line per run).
# Usage: bash tools/gpu_ab_r02e.sh halfwave|split|treestream|inflight|fill
#   halfwave   : half-wave walkers vs SM_NO_HALF_WAVE=1, and their chunk sizes (N=8 view-group share)
#   split      : sm_match_begin/finish vs sm_match_async (--no-split), C2 and the N=8 share
#   treestream : tree stages on a low-priority stream (SM_TREE_STREAM=1) vs one stream
#   inflight   : frames in flight x GPU_MAX_HW_QUEUES
#   fill       : walker fill targets (SM_WALK_FILL / SM_WALK_FILL_DN)
# Each mode first runs the -m gpu parity suite except inflight and fill (env knobs only).
set -o pipefail
MODE=$1
O=gpurun_out/ab_$MODE; mkdir -p $O
VD="--emulate-rank 0/8 --shard vd"
run() {  # name, env assignments, bench args
  env $2 timeout -k 10 200 python bench.py --steps 16 --warmup 4 --no-cpu --no-host-io $3 > $O/$1.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('$O/$1.log').read().strip().splitlines()[-1]);print('%-12s %.3f ms/frame lat %.3f' % ('$1', d['ms_per_step'], d['latency_ms_per_frame']), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
}
suite() {
  timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "tests exit $rc" >> $O/tests.log; tail -2 $O/tests.log
  [ $rc -eq 0 ] || exit $rc
}
case $MODE in
  halfwave)
    suite
    EXP_BENCH_ARGS="$VD" bash tools/gpu_exp.sh dn2 "-DWALK_DN_CHH=2" dn3 "-DWALK_DN_CHH=3" up2 "-DWALK_UP_CHH=2" up4 "-DWALK_UP_CHH=4" || exit 4
    for r in 1 2; do run full.$r "SM_NO_HALF_WAVE=1" "$VD"; run half.$r "X=1" "$VD"; done ;;
  split)
    suite
    for r in 1 2; do
      run c2_async.$r "X=1" "--no-split"; run c2_split.$r "X=1" ""
      run vd8_async.$r "X=1" "$VD --no-split"; run vd8_split.$r "X=1" "$VD"
    done ;;
  treestream)
    suite
    for r in 1 2; do
      run c2_one.$r "SM_TREE_STREAM=0" ""; run c2_ts.$r "SM_TREE_STREAM=1" ""
      run c2_ts_q8.$r "SM_TREE_STREAM=1 GPU_MAX_HW_QUEUES=8" ""
      run vd8_one.$r "SM_TREE_STREAM=0" "$VD"; run vd8_ts.$r "SM_TREE_STREAM=1" "$VD"
      run vd8_ts_q8.$r "SM_TREE_STREAM=1 GPU_MAX_HW_QUEUES=8" "$VD"
    done ;;
  inflight)
    for q in 4 8 16; do for f in 3 4 6; do run vd_q${q}_f$f "GPU_MAX_HW_QUEUES=$q" "$VD --inflight $f"; done; done
    for q in 4 8; do for f in 3 4; do run c2_q${q}_f$f "GPU_MAX_HW_QUEUES=$q" "--inflight $f"; done; done ;;
  fill)
    for r in 1 2; do
      run base.$r "X=1" "$VD"; run f16k.$r "SM_WALK_FILL=16384 SM_WALK_FILL_DN=16384" "$VD"
      run f32k.$r "SM_WALK_FILL=32768 SM_WALK_FILL_DN=32768" "$VD"; run f4k.$r "SM_WALK_FILL=4096 SM_WALK_FILL_DN=4096" "$VD"
    done ;;
  *) echo "unknown mode $MODE"; exit 2 ;;
esac
