# One GPU session (edited per session; logs under gpurun_out/s/)
# This session: the up chain's per-launch spans and the chain wave's wait / compute split at C2, from
# prebuilt diagnostic libraries (variants/ct: -DSM_CHAIN_TIMES, variants/prof: -DSM_CHAIN_PROF).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s
SM_LIB=$GRAFT_REPO_ROOT/variants/ct/libstereomst.so timeout -k 10 300 python tools/chain_prof_run.py > gpurun_out/s/chain_times.log 2>&1 || exit 2
python tools/chain_times.py gpurun_out/s/chain_times.log > gpurun_out/s/chain_times.txt || exit 3
grep -E "total span|repair|wait" gpurun_out/s/chain_times.txt
SM_LIB=$GRAFT_REPO_ROOT/variants/prof/libstereomst.so timeout -k 10 300 python tools/chain_prof_run.py > gpurun_out/s/chain_prof.log 2>&1 || exit 4
grep -E "^up chain" gpurun_out/s/chain_prof.log | sort -t' ' -k6 -n -r | head -12 || true
# the driver's bench command under a kernel trace: the timed region's launches against the line's HIP events
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/s/drv -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s/drv_bench.log 2>&1 || exit 5
python tools/timed_region.py gpurun_out/s/drv/run_kernel_trace.csv gpurun_out/s/drv_bench.log > gpurun_out/s/timed_region.txt 2>&1 || exit 6
grep -h '^{' gpurun_out/s/drv_bench.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());r=d['roofline'];print('same run: %.3f ms/frame, HIP events: %s avg %.1f us' % (d['ms_per_step'], r['kernel'], r['avg_launch_ms'] * 1e3))" >> gpurun_out/s/timed_region.txt || true
cat gpurun_out/s/timed_region.txt
rm -f gpurun_out/s/drv/run_kernel_trace.csv.gz
