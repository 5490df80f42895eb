# round 4: chain kernel with batched LDS reads, two workgroups per CU; chain threshold sweep -> gpurun_out/r04j
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/test_pms_gpu.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for cm in 96 192 384; do
  SM_PMS_CHAIN_MIN=$cm timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 2 > $O/pms100_cm$cm.log 2>&1 || exit 2
  echo "chain_min $cm: $(tail -1 $O/pms100_cm$cm.log | cut -c1-420)"
done
SM_PMS_SEQ_VIEWS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/raw -o run --output-format csv -- python3 tools/pms_bench.py 1920 1200 128 20 --reps 1 > $O/prof.log 2>&1 || exit 5
f=$(find $O/raw -name '*kernel_trace.csv' | head -1)
cp "$f" $O/kernel_trace_pms20_seq.csv
