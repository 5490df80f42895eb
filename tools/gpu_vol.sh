set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "volume or mccnn" > gpurun_out/tv.log 2>&1
rc=$?; echo "vol tests exit $rc"; tail -3 gpurun_out/tv.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tall.log 2>&1
rc=$?; echo "all gpu tests exit $rc"; tail -2 gpurun_out/tall.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bv.log 2>&1; echo "bench $?"
