# Kernel trace of segment mode with 3 frames in flight (GPU busy fraction, per-family time) -> gpurun_out/segtrace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/segtrace
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/raw -o run --output-format csv -- python3 bench.py --segment-c 5000 --no-cpu --no-pms --no-host-io --steps 12 --warmup 3 > $O/bench.log 2>&1 || exit 1
f=$(find $O/raw -name '*kernel_trace.csv' | head -1)
cp "$f" $O/kernel_trace.csv
