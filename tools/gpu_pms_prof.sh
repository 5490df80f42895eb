# MST_PMS kernel statistics (C2, 10 calls per view) -> gpurun_out/pmsprof
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmsprof
mkdir -p $O
timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 10 --reps 1 > $O/plain.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/raw -o run --output-format csv -- python3 tools/pms_bench.py 1920 1200 128 10 --reps 1 > $O/prof.log 2>&1 || exit 2
f=$(find $O/raw -name '*kernel_stats.csv' | head -1)
cp "$f" $O/kernel_stats.csv
tail -3 $O/plain.log | cut -c1-600
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/kernel_stats.csv')))[:18]:
    print(r['Name'][:60].ljust(60), r['Calls'].rjust(6), '%9.2f ms total' % (float(r['TotalDurationNs'])/1e6), '%8.1f us avg' % (float(r['AverageNs'])/1e3), '%8.1f max' % (float(r['MaxNs'])/1e3))
"
