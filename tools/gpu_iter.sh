# One iteration on the GPU box: full GPU parity suite, bench (3 runs), then the chain-wave
# profile of each build_variants/* (SM_CHAIN_PROF builds) on the C2 match.
set -o pipefail
mkdir -p gpurun_out/it
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/it/tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 gpurun_out/it/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/it/b$i.log 2>&1 || { echo bench FAILED; exit 1; }
  python - gpurun_out/it/b$i.log <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print("ms/frame %.3f" % d['ms_per_step'], {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()}, {k: round(v,3) for k,v in d['stages_ms'].items() if k in ('mst_ms','layout_ms','up_ms','down_ms')})
PY
done
for d in build_variants/prof*/; do
  [ -d "$d" ] || continue
  n=$(basename $d)
  SM_LIB=$PWD/$d/libstereomst.so timeout -k 10 200 python tools/chain_prof_run.py > gpurun_out/it/$n.log 2>&1 || { echo "$n FAILED"; exit 1; }
  echo "== $n"; grep -E "len (1[0-9]{4})" gpurun_out/it/$n.log
done
[ -n "$AB" ] && ROUNDS=2 bash tools/ab_bench.sh
true
