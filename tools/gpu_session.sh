# One GPU session (edited per session; logs under gpurun_out/s/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s
timeout -k 10 900 python -u -m pytest tests/test_pms_gpu.py -x -q --timeout 400 --timeout-method thread > gpurun_out/s/tests_pms.log 2>&1; rc=$?; tail -2 gpurun_out/s/tests_pms.log; [ $rc -eq 0 ] || exit 7
SM_LIB=$GRAFT_REPO_ROOT/variants/base/libstereomst.so timeout -k 10 300 python tools/pms_bench.py 1920 1200 128 100 --reps 2 > gpurun_out/s/pms_base.log 2>&1 || exit 2
timeout -k 10 300 python tools/pms_bench.py 1920 1200 128 100 --reps 2 > gpurun_out/s/pms_new.log 2>&1 || exit 3
for f in base new; do python3 -c "import json;d=json.loads(open('gpurun_out/s/pms_$f.log').read().strip().splitlines()[-1])['gpu'];print('$f frame %.1f ms first %.1f later/view %.2f' % (d['wall_ms'], d['iter0_ms'], d['ms_per_later_call_per_view']))"; done
