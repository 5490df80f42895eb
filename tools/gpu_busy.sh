# Kernel traces of the N=8 view-group share (half-wave on/off) and C2, with the busy analysis.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/busy; mkdir -p $O
B="python bench.py --steps 24 --warmup 3 --no-cpu --no-host-io"
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/vd8 -o run --output-format csv -- $B --emulate-rank 0/8 --shard vd > $O/vd8.log 2>&1 || exit 1
python3 tools/busy.py $O/vd8/run_kernel_trace.csv 0.3 || exit 2
SM_NO_HALF_WAVE=1 timeout -k 10 240 rocprofv3 --kernel-trace -d $O/vd8f -o run --output-format csv -- $B --emulate-rank 0/8 --shard vd > $O/vd8f.log 2>&1 || exit 3
python3 tools/busy.py $O/vd8f/run_kernel_trace.csv 0.3 || exit 4
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/c2 -o run --output-format csv -- $B > $O/c2.log 2>&1 || exit 5
python3 tools/busy.py $O/c2/run_kernel_trace.csv 0.3 || exit 6
