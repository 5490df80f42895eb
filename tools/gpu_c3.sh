set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread -k "full_size_c4" > gpurun_out/tc4.log 2>&1
rc=$?; echo "c4 test $rc"; tail -2 gpurun_out/tc4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --width 3840 --height 2160 --disp 256 --steps 5 --warmup 2 --no-cpu > gpurun_out/bc3.log 2>&1; echo "c3 bench $?"
timeout -k 10 300 python bench.py --disp 256 --steps 10 --warmup 2 --no-cpu > gpurun_out/bc4.log 2>&1; echo "c4 bench $?"
