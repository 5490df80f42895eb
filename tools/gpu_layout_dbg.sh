set -o pipefail
mkdir -p gpurun_out
DBG=SM_LAYOUT_DEBUG timeout -k 10 100 python tools/mst_debug.py > gpurun_out/layout_dbg.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ltrace -o lt -- python bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/ltrace.log 2>&1
