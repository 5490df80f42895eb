set -o pipefail
mkdir -p gpurun_out
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/t_all.log 2>&1
rc=$?; echo "tests exit $rc" >> gpurun_out/t_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/b_default.log 2>&1
