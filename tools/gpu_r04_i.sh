# round 4: PMS chain kernel for long paths: PMS parity suite, 100-call C2 frames (prep phase times on
# stderr), A/B SM_PMS_NO_CHAIN=1, SM_PMS_BIG sweep of the first call, kernel trace -> gpurun_out/r04i
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/test_pms_gpu.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
SM_PREP_DEBUG=1 timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 2 > $O/pms100.log 2>&1 || exit 2
grep pms_build_forest $O/pms100.log | tail -2
tail -1 $O/pms100.log | cut -c1-1500
SM_PMS_NO_CHAIN=1 timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 1 > $O/pms100_nochain.log 2>&1 || exit 3
tail -1 $O/pms100_nochain.log | cut -c1-400
for b in 4096 16384 65536; do
  SM_PMS_BIG=$b timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 2 --reps 2 > $O/pms2_big$b.log 2>&1 || exit 4
  echo "SM_PMS_BIG=$b: $(tail -1 $O/pms2_big$b.log | cut -c1-300)"
done
SM_PMS_SEQ_VIEWS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/raw -o run --output-format csv -- python3 tools/pms_bench.py 1920 1200 128 20 --reps 1 > $O/prof.log 2>&1 || exit 5
f=$(find $O/raw -name '*kernel_trace.csv' | head -1)
cp "$f" $O/kernel_trace_pms20_seq.csv
f=$(find $O/raw -name '*kernel_stats.csv' | head -1)
cp "$f" $O/kernel_stats_pms20_seq.csv
