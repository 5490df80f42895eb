# Round profile set (run on the GPU box): kernel-trace stats of the default bench (frames in flight),
# the same for one frame at a time, two PMC passes, and the default bench with the CPU baseline.
# Outputs under gpurun_out/<tag>/.  Usage: bash tools/gpu_prof_round.sh r02
set -o pipefail
TAG=${1:-r02}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu --no-host-io --no-pms > $O/stats_bench.log 2>&1 || exit 11
python tools/timed_region.py $O/stats/run_kernel_trace.csv $O/stats_bench.log > $O/timed_region.txt 2>&1 || exit 17
grep -h '^{' $O/stats_bench.log | python3 -c "import json,sys;r=json.loads(sys.stdin.read())['roofline'];print('same run, HIP events: %s avg %.1f us' % (r['kernel'], r['avg_launch_ms'] * 1e3))" >> $O/timed_region.txt || true
cat $O/timed_region.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats1 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu --no-host-io --no-pms --inflight 1 > $O/stats1_bench.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu --no-host-io --no-pms --inflight 1 > $O/pmc_fetch.log 2>&1 || exit 13
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu --no-host-io --no-pms --inflight 1 > $O/pmc_write.log 2>&1 || exit 14
python tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write auto $O/pmc_traffic.json > $O/pmc_traffic.log 2>&1 || exit 15
cp $O/pmc_traffic.json profiles/pmc_traffic.json  # the default bench below reports this traffic
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || exit 16
echo done
