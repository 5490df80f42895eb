# Kernel trace of a 10-call MST_PMS frame (C2): per-stream busy time and gaps of the later calls
# (tools/pms_gaps.py).  Output under gpurun_out/pmstrace/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmstrace
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/raw -o run --output-format csv -- python tools/pms_bench.py 1920 1200 128 10 --reps 1 > $O/run.log 2>&1 || exit 1
f=$(find $O/raw -name '*kernel_trace.csv' | head -1)
python tools/pms_gaps.py "$f" > $O/gaps.txt 2>&1 || exit 2
gzip -c "$f" > $O/kernel_trace.csv.gz
rm -rf $O/raw
cat $O/gaps.txt
