# (round 6 experiment; the banded order was measured slower and removed: profiles/r06/ab_xcd_bands/)
# XCD-banded chain blocks: parity subset, interleaved A/B (dev library, SM_NO_XCD_BANDS=1 = the old order),
# and FETCH/WRITE PMC traffic of both orders, one frame at a time (MST only).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06xcd; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -k "piece or cut or repair or c2 or c3 or c4 or one_view or chain or layout or flir or shard" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
D="SM_LIB=stereomatch_amd/libstereomst_dev.so"
REPS=2 bash tools/gpu_ab.sh "c2old|$D SM_NO_XCD_BANDS=1|" "c2band|$D|" "s8old|$D SM_NO_XCD_BANDS=1|--emulate-rank 0/8 --frame-groups 1" "s8band|$D|--emulate-rank 0/8 --frame-groups 1" || exit 3
M="--no-cpu --no-host-io --no-pms --no-segment --steps 2 --warmup 1 --inflight 1"
for var in old band; do
  if [ $var = old ]; then export SM_NO_XCD_BANDS=1; else unset SM_NO_XCD_BANDS; fi
  SM_LIB=stereomatch_amd/libstereomst_dev.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/f_$var -o run --output-format csv -- python bench.py --dev $M > $O/f_$var.log 2>&1 || exit 4
  SM_LIB=stereomatch_amd/libstereomst_dev.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/w_$var -o run --output-format csv -- python bench.py --dev $M > $O/w_$var.log 2>&1 || exit 5
  python tools/pmc_traffic.py $O/f_$var $O/w_$var auto $O/pmc_$var.json > $O/pmc_$var.log 2>&1 || exit 6
  python3 -c "import json;d=json.load(open('$O/pmc_$var.json'));print('$var', {k:round(v['hbm_bytes_per_frame']/1e9,3) for k,v in d.items() if isinstance(v,dict) and 'chain' in k})"
done
echo done
