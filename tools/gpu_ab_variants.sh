# A/B of build_variants/* (non-prof) on one box + chain profile of build_variants/prof_*; ROUNDS alternations
set -o pipefail
mkdir -p gpurun_out/abv
for d in build_variants/prof_*/; do
  [ -d "$d" ] || continue
  SM_LIB=$PWD/$d/libstereomst.so timeout -k 10 200 python tools/chain_prof_run.py > gpurun_out/abv/$(basename $d).log 2>&1 || { echo "prof FAILED"; exit 1; }
  echo "== $(basename $d)"; grep -E "len (1[0-9]{4})" gpurun_out/abv/$(basename $d).log
done
for i in $(seq 1 ${ROUNDS:-2}); do for d in build_variants/*/; do
  n=$(basename $d); case $n in prof_*) continue;; esac
  SM_LIB=$PWD/$d/libstereomst.so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/abv/$n.$i 2>&1 || { echo "$n FAILED"; exit 1; }
  python - gpurun_out/abv/$n.$i $n <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], "ms/frame %.3f" % d['ms_per_step'], {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()})
PY
done; done
