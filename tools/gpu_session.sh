set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g2
timeout -k 10 400 python -u -m pytest tests/test_pms_gpu.py -k "forest_matches_host_build or golden_bitexact or many_trees" -x -q --timeout 200 --timeout-method thread > gpurun_out/g2/tests_forest.log 2>&1; rc=$?; tail -3 gpurun_out/g2/tests_forest.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python tools/pms_bench.py 1920 1200 128 100 --reps 1 > gpurun_out/g2/pms100.log 2>&1 || exit 4
tail -2 gpurun_out/g2/pms100.log | cut -c1-900
REPS=2 bash tools/gpu_ab.sh "base||" "skm|SM_EXP_SKIP=mst|" "skl|SM_EXP_SKIP=layout|" "fo|SM_EXP_FILTER_ONLY=1|"
