# Kernel statistics of segment mode (GPU segmentation) -> gpurun_out/segprof/<R>/kernel_stats.csv
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for R in ${ROUNDS:-2}; do
  O=gpurun_out/segprof/r$R
  mkdir -p $O
  SM_SEG_GLOBAL_ROUNDS=$R timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/raw -o run --output-format csv -- python3 bench.py --segment-c 5000 --no-cpu --no-pms --steps 3 --warmup 1 --inflight 1 > $O/bench.log 2>&1 || exit 1
  f=$(find $O/raw -name '*kernel_stats.csv' | head -1)
  cp "$f" $O/kernel_stats.csv
  echo "== R=$R"; head -14 $O/kernel_stats.csv | cut -d, -f1-5 | cut -c1-120
  python3 -c "import json;d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],3), d['stages_ms']['mst_ms'])"
done
