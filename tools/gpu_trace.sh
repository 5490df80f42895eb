# per-dispatch kernel trace of a short bench run (rocprofv3), summaries under gpurun_out/$1
set -o pipefail
OUT=${1:-trace}
mkdir -p gpurun_out/$OUT
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$OUT -o run --output-format csv -- python bench.py --steps ${2:-2} --warmup 1 --no-cpu > gpurun_out/$OUT/bench.log 2>&1
echo "prof exit $?"
