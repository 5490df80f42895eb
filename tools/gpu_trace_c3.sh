# kernel stats of the C3 workload (3840x2160, D=256) under rocprofv3
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-trc3}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python bench.py --width 3840 --height 2160 --disp 256 --steps 2 --warmup 1 --no-cpu > $O/bench.log 2>&1
echo "prof exit $?"
