set -o pipefail
mkdir -p gpurun_out/prof1
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof1/bench.log 2>&1
echo "prof exit $?"
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "full_size or flir_c1" > gpurun_out/t2.log 2>&1
echo "tests exit $?"
