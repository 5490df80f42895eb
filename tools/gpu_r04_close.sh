# Close of round 4 (two gpurun calls): "final" = smoke, the -m gpu suite, the default bench and a batch line
# (tools/gpu_final.sh); "prof" = the profile set of this build (tools/gpu_prof_round.sh r04) and a rocprof
# kernel summary of the 100-call MST_PMS frame.  Usage: bash tools/gpu_r04_close.sh final|prof
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
case "$1" in
final)
  bash tools/gpu_final.sh || exit 2
  timeout -k 10 300 python bench.py --segment-c 5000 --min-size 200 --no-cpu --no-pms > gpurun_out/final/bench_segment.log 2>&1 || exit 5
  python3 -c "import json;d=json.loads(open('gpurun_out/final/bench_segment.log').read().strip().splitlines()[-1]);print('segment', round(d['ms_per_step'],3), 'latency', round(d['latency_ms_per_frame'],2))"
  ;;
prof)
  bash tools/gpu_prof_round.sh r04 || exit 3
  O=gpurun_out/r04
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pmsraw -o run --output-format csv -- python3 tools/pms_bench.py 1920 1200 128 100 --reps 1 > $O/pms100_prof.log 2>&1 || exit 4
  f=$(find $O/pmsraw -name '*kernel_stats.csv' | head -1); cp "$f" $O/pms100_kernel_stats.csv
  rm -rf $O/pmsraw
  tail -1 $O/pms100_prof.log | cut -c1-600
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/segraw -o run --output-format csv -- python3 bench.py --segment-c 5000 --min-size 200 --inflight 1 --steps 4 --warmup 2 --no-cpu --no-pms --no-host-io > $O/seg1_prof.log 2>&1 || exit 6
  f=$(find $O/segraw -name '*kernel_stats.csv' | head -1); cp "$f" $O/seg1_kernel_stats.csv
  rm -rf $O/segraw
  echo seg traced
  ;;
*) echo "usage: $0 final|prof"; exit 1 ;;
esac
