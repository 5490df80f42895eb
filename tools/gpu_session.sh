# One GPU session (edited per session; logs under gpurun_out/s/)
# This session: the driver's own bench command on HEAD (final build), one run.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s/driver_cmd.log 2>&1 || exit 2
grep -h '^{' gpurun_out/s/driver_cmd.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['end_to_end']['frac'], d['roofline']['traffic_source']['same_build'])"
