set -o pipefail
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t_all.log 2>&1
rc=$?; tail -1 gpurun_out/t_all.log; [ $rc -eq 0 ] || exit $rc
SM_LIB=$PWD/build_variants/prof_pipe/libstereomst.so timeout -k 10 200 python tools/chain_prof_run.py > gpurun_out/pp.log 2>&1 || exit 1
grep -E "len (1[0-9]{4})" gpurun_out/pp.log
mkdir -p gpurun_out/ab
for i in 1 2 3; do for d in pipe nopipe; do
  SM_LIB=$PWD/build_variants/$d/libstereomst.so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/ab/$d.$i 2>&1 || { echo "$d FAILED"; exit 1; }
  python - gpurun_out/ab/$d.$i $d <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], "ms/frame %.3f" % d['ms_per_step'], {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()})
PY
done; done
