# Per-round launch times of the filter for a few shares (tools/round_probe.py under a kernel trace).
# Usage (on the box): bash tools/gpu_rounds.sh <tag>  -> gpurun_out/<tag>/rounds_*.txt
set -o pipefail
TAG=${1:-rounds}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for spec in "share8:--views 1 --D 64 --d0 0 --dtotal 256" "c2:--views 3 --D 128 --dtotal 128" "d8:--views 3 --D 32 --d0 0 --dtotal 256"; do
  n=${spec%%:*}; a=${spec#*:}
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$n -o run -- python tools/round_probe.py $a > $O/probe_$n.log 2>&1 || exit 1
  python tools/round_split.py $O/tr_$n/run_kernel_trace.csv $O/probe_$n.log > $O/rounds_$n.txt 2>&1 || exit 2
  tail -4 $O/rounds_$n.txt
done
echo done
