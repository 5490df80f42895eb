# Final check of a round: smoke(), the -m gpu suite, the default bench and one C5 (batch) line.
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || exit 1
tail -2 gpurun_out/final/smoke.log
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/final/tests.log 2>&1 || exit 2
tail -1 gpurun_out/final/tests.log
timeout -k 10 400 python bench.py > gpurun_out/final/bench_default.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --mode batch --steps 6 --warmup 2 --no-cpu > gpurun_out/final/bench_batch.log 2>&1 || exit 4
for f in bench_default bench_batch; do
  python3 -c "import json;d=json.loads(open('gpurun_out/final/$f.log').read().strip().splitlines()[-1]);print('$f', d['config']['workload'], round(d['ms_per_step'],3), '%.4g' % d['value'], round(d['roofline']['frac'],3))"
done
