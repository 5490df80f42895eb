# round 6 A/B 11: compact rows with coordinate-based row lookup in k_meta vs the committed build (C2, N=8 share)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ab11
mkdir -p $O
timeout -k 10 300 python tools/layout_check.py > $O/layout_check.log 2>&1 || { cat $O/layout_check.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 2; }
H=SM_LIB=variants/head/libstereomst.so
E="--emulate-rank 0/8 --frame-groups 1"
REPS=3 bash tools/gpu_ab.sh "head|$H|" "new||" "head_share|$H|$E" "new_share||$E" || exit 3
echo done
