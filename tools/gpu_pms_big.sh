# MST_PMS first-call sweep of the big-tree threshold (SM_PMS_BIG): 2-call frames, 2 reps each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmsbig
mkdir -p $O
for big in 1024 256 512 2048 4096; do
  SM_PMS_BIG=$big timeout -k 10 300 python tools/pms_bench.py 1920 1200 128 2 --reps 2 > $O/big_$big.log 2>&1 || exit 2
  python3 -c "import json;d=json.loads(open('$O/big_$big.log').read().strip().splitlines()[-1])['gpu'];print('big $big first call %.1f ms (views %s)' % (d['iter0_ms'], [round(x,1) for x in d['first_ms_view']]))"
done
