# GPU segmentation check: segment-mode parity tests, then segment-mode bench lines (3 and 6 in flight).
set -o pipefail
O=gpurun_out/seg
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "segment or pms" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --segment-c 5000 --no-cpu --no-pms --steps 10 --warmup 2 > $O/bench_seg.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --segment-c 5000 --no-cpu --no-pms --steps 12 --warmup 3 --inflight 6 > $O/bench_seg6.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --no-cpu --steps 6 --warmup 2 > $O/bench_pms.log 2>&1 || exit 5
for f in bench_seg bench_seg6 bench_pms; do
  python3 -c "import json;d=json.loads(open('$O/$f.log').read().strip().splitlines()[-1]);print('$f', round(d['ms_per_step'],3), d['config']['tree'], d['stages_ms'], (d.get('pms') or {}).get('host_prep_ms'), (d.get('pms') or {}).get('first_call_ms_per_view'))"
done
