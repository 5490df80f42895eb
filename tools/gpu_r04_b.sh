# round 4: concurrent-view MST_PMS + evaluation counters, the executed shim, the multi-context segment
# test; then the 100-call C2 frame, concurrent views vs SM_PMS_SEQ_VIEWS=1 -> gpurun_out/r04b
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/test_pms_gpu.py \
  tests/test_shim_gpu.py "tests/test_gpu_parity.py::test_segment_mode_begin_on_many_contexts_bitexact" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 2 > $O/pms100.log 2>&1 || exit 2
tail -1 $O/pms100.log | cut -c1-1500
SM_PMS_SEQ_VIEWS=1 timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 1 > $O/pms100_seq.log 2>&1 || exit 3
tail -1 $O/pms100_seq.log | cut -c1-1500
