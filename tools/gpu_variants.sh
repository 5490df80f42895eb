# timing probes: per-round walker times for SM_WALK_VARIANT = 0 1 2 (product path is 0)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for v in 0 1 2; do
  mkdir -p gpurun_out/var$v
  SM_WALK_VARIANT=$v timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/var$v -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/var$v/bench.log 2>&1 || exit 1
done
echo done
