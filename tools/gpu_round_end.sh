# End-of-round measurement set: rocprof profile set (tools/gpu_prof_round.sh), C3 and C4 benches,
# per-rank shares of the strong-mode partitions (tools/gpu_emulate.sh).
# Usage (on the box): bash tools/gpu_round_end.sh r02e
set -o pipefail
TAG=${1:-r02e}
bash tools/gpu_prof_round.sh $TAG || exit $?
O=gpurun_out/$TAG
timeout -k 10 300 python bench.py --width 3840 --height 2160 --disp 256 --steps 6 --warmup 2 --no-cpu > $O/bench_c3.log 2>&1 || exit 21
timeout -k 10 300 python bench.py --disp 256 --steps 12 --warmup 3 --no-cpu > $O/bench_c4.log 2>&1 || exit 22
bash tools/gpu_emulate.sh || exit 23
echo round-end done
