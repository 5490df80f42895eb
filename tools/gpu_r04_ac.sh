# round 4: segment mode -- k_seg_small per-bucket timings (SM_SEG_PROF) -> gpurun_out/r04ac
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ac
mkdir -p $O
SM_SEG_PROF=1 timeout -k 10 300 python3 bench.py --segment-c 5000 --min-size 200 --inflight 1 --steps 2 --warmup 1 --no-cpu --no-pms > $O/prof.log 2>&1 || exit 1
grep "seg prof" $O/prof.log | tail -2 | cut -c1-1500
SM_SEG_PROF=1 SM_SEG_NOSPLIT=1 timeout -k 10 300 python3 bench.py --segment-c 5000 --min-size 200 --inflight 1 --steps 2 --warmup 1 --no-cpu --no-pms > $O/prof_nosplit.log 2>&1 || exit 2
grep "seg prof" $O/prof_nosplit.log | tail -2 | cut -c1-1500
