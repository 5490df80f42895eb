# GPU parity suite, then A/B of the contracted vs pixel Boruvka rounds on one box.
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t_all.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 gpurun_out/t_all.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/ab/c.$i 2>&1 || { echo c FAILED; exit 1; }
  SM_MST_PIXEL_ROUNDS=1 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/ab/p.$i 2>&1 || { echo p FAILED; exit 1; }
  echo "contract $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/c.$i) $(grep -o '"mst[^,]*' gpurun_out/ab/c.$i | head -1)"
  echo "pixel    $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/p.$i) $(grep -o '"mst[^,]*' gpurun_out/ab/p.$i | head -1)"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mstprof -o mst -- python bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/mstprof.log 2>&1 || { echo prof FAILED; exit 1; }
find gpurun_out/mstprof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/mst_kernel_stats.csv
