# GPU parity suite, then A/B of the merged chain launches vs SM_NO_MERGE on one box
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t_all.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 gpurun_out/t_all.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for m in merge nomerge; do
    if [ $m = nomerge ]; then export SM_NO_MERGE=1; else unset SM_NO_MERGE; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/ab/$m.$i 2>&1 || { echo "$m FAILED"; exit 1; }
    python - gpurun_out/ab/$m.$i $m <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], "ms/frame %.3f" % d['ms_per_step'], {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()}, {k: round(v,3) for k,v in d['stages_ms'].items() if k in ('up_ms','down_ms')})
PY
  done
done
