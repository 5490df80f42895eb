# One GPU session (edited per session; logs under gpurun_out/s/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s
timeout -k 10 300 python tools/host_probe.py 40 > gpurun_out/s/host_probe.log 2>&1 || exit 2
timeout -k 10 300 python tools/host_probe.py 40 >> gpurun_out/s/host_probe.log 2>&1 || exit 2
cat gpurun_out/s/host_probe.log
bash tools/gpu_pms_big.sh || exit 3
