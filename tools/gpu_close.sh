# Close of a round on one GPU box: smoke(), the full -m gpu suite, the profile set of this build
# (kernel stats in flight and one frame at a time, FETCH_SIZE / WRITE_SIZE PMC passes ->
# profiles/pmc_traffic.json), the default bench line (which then reports same_build: true), the
# 100-call MST_PMS frame, and the N = 8 per-rank emulations.  Outputs under gpurun_out/<tag>/.
# Usage (on the box): bash tools/gpu_close.sh r05 [skip-tests]
set -o pipefail
TAG=${1:-close}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -2 $O/smoke.log
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests_gpu.log 2>&1 || { tail -5 $O/tests_gpu.log; exit 2; }
  tail -1 $O/tests_gpu.log
fi
bash tools/gpu_prof_round.sh $TAG || exit 3
python3 -c "import json;d=json.loads(open('$O/bench_default.log').read().strip().splitlines()[-1]);print('default', round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],3), 'same_build', d['roofline'].get('traffic_source',{}).get('same_build'))" || true
timeout -k 10 300 python tools/pms_bench.py 1920 1200 128 100 --reps 2 > $O/pms100.log 2>&1 || exit 4
tail -1 $O/pms100.log | cut -c1-200
timeout -k 10 300 python bench.py --disp 256 --steps 20 --warmup 5 --no-cpu --no-host-io --no-pms --no-segment > $O/c4_1gpu.log 2>&1 || exit 6
python3 -c "import json;d=json.loads(open('$O/c4_1gpu.log').read().strip().splitlines()[-1]);print('C4 on 1 GPU', round(d['ms_per_step'],3))" || true
for spec in "0/8 --frame-groups 1" "0/8 --frame-groups 2" "0/8 --shard d --frame-groups 1"; do
  set -- $spec
  tagn=$(echo "$spec" | tr ' /' '__' | tr -d '-')
  timeout -k 10 300 python bench.py --emulate-rank $spec --steps 20 --warmup 5 --no-cpu --no-host-io --no-pms --no-segment > $O/emu_$tagn.log 2>&1 || exit 5
  python3 -c "import json;d=json.loads(open('$O/emu_$tagn.log').read().strip().splitlines()[-1]);print('emu $spec', round(d['ms_per_step'],3), d['config'].get('workload'))" || true
done
echo done
