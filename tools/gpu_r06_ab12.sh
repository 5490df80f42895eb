# round 6 A/B 12: piece repair statistics (committed build vs product) and C2 after hoisting k_meta's row loads
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ab12
mkdir -p $O
timeout -k 10 300 python tools/layout_check.py > $O/layout_check.log 2>&1 || { cat $O/layout_check.log; exit 1; }
SM_LIB=variants/head/libstereomst.so timeout -k 10 120 python tools/piece_stats.py > $O/pieces_head.log 2>&1 || exit 2
timeout -k 10 120 python tools/piece_stats.py > $O/pieces_new.log 2>&1 || exit 3
grep -h pieces $O/pieces_head.log; echo ---; grep -h pieces $O/pieces_new.log
H=SM_LIB=variants/head/libstereomst.so
REPS=3 bash tools/gpu_ab.sh "head|$H|" "new||" || exit 4
echo done
