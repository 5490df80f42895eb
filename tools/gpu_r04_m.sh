# round 4: the GPU schedule forest (sm_pms_forest.hip) checked against the host build, the PMS suite, the
# 100-call C2 frame (GPU vs host forest), chain threshold sweep, kernel trace -> gpurun_out/r04m
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_pms_gpu.py \
  -k "gpu_forest_matches" > $O/tests_forest.log 2>&1 || { tail -40 $O/tests_forest.log; exit 1; }
tail -3 $O/tests_forest.log
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/test_pms_gpu.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 2 > $O/pms100.log 2>&1 || exit 2
tail -1 $O/pms100.log | cut -c1-1500
SM_PMS_HOST_FOREST=1 timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 2 > $O/pms100_hostforest.log 2>&1 || exit 3
echo "host forest: $(tail -1 $O/pms100_hostforest.log | cut -c1-420)"
for cm in 192 384; do
  SM_PMS_CHAIN_MIN=$cm timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 2 > $O/pms100_cm$cm.log 2>&1 || exit 4
  echo "chain_min $cm: $(tail -1 $O/pms100_cm$cm.log | cut -c1-420)"
done
SM_PMS_SEQ_VIEWS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/raw -o run --output-format csv -- python3 tools/pms_bench.py 1920 1200 128 20 --reps 1 > $O/prof.log 2>&1 || exit 5
f=$(find $O/raw -name '*kernel_trace.csv' | head -1)
cp "$f" $O/kernel_trace_pms20_seq.csv
f=$(find $O/raw -name '*kernel_stats.csv' | head -1)
cp "$f" $O/kernel_stats_pms20_seq.csv
