# smoke + the -m gpu suite (the degenerate-tree file last), logs under gpurun_out/<tag>/
set -o pipefail
TAG=${1:-tests}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread --deselect tests/test_degenerate_trees.py ${EXTRA:-} > $O/tests_gpu.log 2>&1 || { tail -30 $O/tests_gpu.log; exit 2; }
tail -1 $O/tests_gpu.log
timeout -k 10 900 python -u -m pytest tests/test_degenerate_trees.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests_degenerate.log 2>&1 || { tail -30 $O/tests_degenerate.log; exit 3; }
tail -8 $O/tests_degenerate.log
echo done
