# Context memory at C3 / C2 after the segment-aggregate sizing fix, and the C3 / cut-path parity tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06mem; mkdir -p $O
timeout -k 10 300 python tools/mem_probe.py 3840 2160 256 > $O/mem_c3.log 2>&1 || exit 1
timeout -k 10 300 python tools/mem_probe.py 1920 1200 128 > $O/mem_c2.log 2>&1 || exit 2
grep -h context $O/mem_c3.log $O/mem_c2.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -k "c3 or piece or cut or repair or one_view or c4" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 3; }
tail -2 $O/tests.log
