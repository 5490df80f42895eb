# quick iteration: parity subset, then two default bench runs (kernel and stage breakdown)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${1:-match_bitexact or aggregate or cost_volume or full_size or flir or pieces_match or layout}" > gpurun_out/tq.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 gpurun_out/tq.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bq$i.log 2>&1 || exit 1; done
python - <<'P'
import json
for i in (1, 2):
    d = json.loads([l for l in open('gpurun_out/bq%d.log' % i) if l.startswith('{')][-1])
    print('%.3f ms' % d['ms_per_step'], {k: round(v, 3) for k, v in d['stages_ms'].items()})
P
