# round 4: planned walks + parallel piece repair: PMS parity suite (incl. forced sequential repair), 100-call
# C2 frame, A/B against SM_PMS_SEQ_REPAIR=1, kernel trace of 20 calls (views in sequence) -> gpurun_out/r04e
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/test_pms_gpu.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 2 > $O/pms100.log 2>&1 || exit 2
tail -1 $O/pms100.log | cut -c1-1500
SM_PMS_NO_CHAIN=1 timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 1 > $O/pms100_nochain.log 2>&1 || exit 3
tail -1 $O/pms100_nochain.log | cut -c1-1500
SM_PMS_SEQ_VIEWS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/raw -o run --output-format csv -- python3 tools/pms_bench.py 1920 1200 128 20 --reps 1 > $O/prof.log 2>&1 || exit 4
f=$(find $O/raw -name '*kernel_trace.csv' | head -1)
cp "$f" $O/kernel_trace_pms20_seq.csv
