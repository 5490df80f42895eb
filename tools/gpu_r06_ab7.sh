# round 6 A/B 7: compact A rows (tile-aggregated row atomics) against the committed build (variants/head)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ab7
mkdir -p $O
H=SM_LIB=variants/head/libstereomst.so
E="--emulate-rank 0/8 --frame-groups 1"
REPS=3 bash tools/gpu_ab.sh "head|$H|" "new||" "head_share|$H|$E" "new_share||$E" || exit 3
P="--dev --steps 5 --warmup 2 --no-cpu --no-host-io --no-pms --no-segment --inflight 1"
SM_LIB=variants/head/libstereomst.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_head -o run -- python bench.py $P > $O/prof_head.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_new -o run -- python bench.py $P > $O/prof_new.log 2>&1 || exit 5
for v in head new; do echo "== $v"; f=$(find $O/prof_$v -name "*kernel_stats.csv" | head -1); python3 -c "
import csv,sys
r=list(csv.DictReader(open('$f')))
for x in r:
    n=x['Name']
    if any(k in n for k in ('k_meta','k_headfix','k_newslot','k_path_emit','k_long_seg','k_down_walk','k_up_walk','k_down_chain','k_up_chain')): print('%-60s %6s %10.1f' % (n[:60], x['Calls'], float(x['AverageNs'])/1e3))
"; done
echo done
