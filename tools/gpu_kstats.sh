# rocprofv3 kernel stats of a short bench run; prints per-frame time of the top kernels
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/ks && mkdir -p gpurun_out/ks
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks -o run -- python bench.py --steps 4 --warmup 1 --no-cpu > gpurun_out/ks/bench.log 2>&1 || exit 1
python - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/ks/**/run_kernel_stats.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows[:40]:
    print("%-44s %7.1f us/frame  %6.1f calls/frame  avg %7.1f us" % (r['Name'][:44], float(r['TotalDurationNs'])/5e3, int(r['Calls'])/5, float(r['AverageNs'])/1e3))
PY
