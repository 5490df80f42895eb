# round 4, first GPU call: the new full-size speculative MST_PMS tests, then a 100-call C2 MST_PMS frame
# (plain and under rocprofv3 --kernel-trace --stats) -> gpurun_out/r04a
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_pms_gpu.py -m gpu \
  -k "full_c2_speculative or flir_c1_two_calls" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -4 $O/tests.log
timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 1 > $O/pms100.log 2>&1 || exit 2
tail -1 $O/pms100.log | cut -c1-800
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/raw -o run --output-format csv -- python3 tools/pms_bench.py 1920 1200 128 100 --reps 1 > $O/prof.log 2>&1 || exit 3
f=$(find $O/raw -name '*kernel_stats.csv' | head -1)
cp "$f" $O/kernel_stats_pms100.csv
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/kernel_stats_pms100.csv')))[:16]:
    print(r['Name'][:60].ljust(60), r['Calls'].rjust(7), '%9.2f ms total' % (float(r['TotalDurationNs'])/1e6), '%8.1f us avg' % (float(r['AverageNs'])/1e3))
"
