# MST_PMS parity tests, then per-call timings with and without the propagation-label dedupe (C2, 10 calls)
set -o pipefail
O=gpurun_out/pmsab
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "pms" --timeout 400 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 10 --reps 2 > $O/dedupe.log 2>&1 || exit 2
SM_PMS_NODEDUP=1 timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 10 --reps 2 > $O/nodedupe.log 2>&1 || exit 3
for f in dedupe nodedupe; do echo $f; tail -1 $O/$f.log | cut -c1-400; done
