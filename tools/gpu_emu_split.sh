# N = 8 per-rank share (rank 0 of 8, one view, 64 slices, every rank on every frame): the share as is,
# with the layout skipped, and with every tree stage skipped (re-filtering the previous tree), so the
# tree stages' part of the share is measured.  Logs under gpurun_out/emu/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/emu
mkdir -p $O
for spec in "base||" "skl|SM_EXP_SKIP=layout|" "fo|SM_EXP_FILTER_ONLY=1|"; do
  label=${spec%%|*}; rest=${spec#*|}; envs=${rest%%|*}
  env $envs timeout -k 10 300 python bench.py --emulate-rank 0/8 --frame-groups 1 --steps 20 --warmup 5 --no-cpu --no-host-io --no-pms --no-segment > $O/$label.log 2>&1 || { echo "FAILED $label"; tail -3 $O/$label.log; exit 2; }
  python3 -c "import json,sys;d=json.loads(open('$O/$label.log').read().strip().splitlines()[-1]);print('$label', round(d['ms_per_step'],3), round(d['latency_ms_per_frame'],2), {a: round(b,3) for a,b in d['kernels_ms_per_step'].items()})"
done
