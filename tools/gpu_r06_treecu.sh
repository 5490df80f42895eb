# (round 6 experiment: the CU-masked tree stream was slower at every mask and was removed; profiles/r06/ab_tree_cumask/)
# Tree stages on a CU-masked stream (dev library, SM_TREE_CUS=n): smoke and the C2 / C1 match tests through the
# dev library with the stream on, then interleaved A/B at C2 and on the N = 8 G = 1 share
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06treecu; mkdir -p $O
export SM_LIB=$GRAFT_REPO_ROOT/stereomatch_amd/libstereomst_dev.so
SM_TREE_CUS=64 timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
SM_TREE_CUS=64 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c2 or flir or c3" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 2; }
tail -1 $O/tests.log
unset SM_LIB
D="SM_LIB=stereomatch_amd/libstereomst_dev.so"
REPS=2 bash tools/gpu_ab.sh "base|$D|" "cu32|$D SM_TREE_CUS=32|" "cu64|$D SM_TREE_CUS=64|" "cu128|$D SM_TREE_CUS=128|" \
  "s8base|$D|--emulate-rank 0/8 --frame-groups 1" "s8cu64|$D SM_TREE_CUS=64|--emulate-rank 0/8 --frame-groups 1"
