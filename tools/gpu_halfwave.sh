# Half-wave down walker: parity suite, then per-rank N=8 view-group share A/B (chunk sizes, and
# the full-wave walker via SM_NO_HALF_WAVE), then the default C2 bench.
# Usage (on the box): bash tools/gpu_halfwave.sh [pytest -k expr]
set -o pipefail
mkdir -p gpurun_out
K="${1:-}"
if [ -n "$K" ]; then
  timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -k "$K" > gpurun_out/t_hw.log 2>&1
else
  timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/t_hw.log 2>&1
fi
rc=$?; echo "tests exit $rc" >> gpurun_out/t_hw.log; tail -3 gpurun_out/t_hw.log
[ $rc -eq 0 ] || exit $rc
EXP_BENCH_ARGS="--emulate-rank 0/8 --shard vd" bash tools/gpu_exp.sh dn2 "-DWALK_DN_CHH=2" dn3 "-DWALK_DN_CHH=3" up2 "-DWALK_UP_CHH=2" up4 "-DWALK_UP_CHH=4" || exit 4
B="python bench.py --steps 10 --warmup 3 --no-cpu --no-host-io --emulate-rank 0/8 --shard vd"
for r in 1 2; do
  SM_NO_HALF_WAVE=1 timeout -k 10 200 $B > gpurun_out/hw_off.log 2>&1 || exit 5
  python3 -c "import json;d=json.loads(open('gpurun_out/hw_off.log').read().strip().splitlines()[-1]);print('full-wave', round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
  timeout -k 10 200 $B > gpurun_out/hw_on.log 2>&1 || exit 6
  python3 -c "import json;d=json.loads(open('gpurun_out/hw_on.log').read().strip().splitlines()[-1]);print('half-wave', round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
done
