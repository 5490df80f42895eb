# A/B of the CU-masked chain stream (SM_CU_CHAIN=k): C2 frame and the N = 8 rank-0
# share, default vs k CUs for the chains.  Usage (on the box): bash tools/gpu_cu_split.sh "0 32 64"
set -o pipefail
O=gpurun_out/cusplit
mkdir -p $O
B="python bench.py --steps 20 --warmup 3 --no-cpu --no-host-io --no-pms"
for k in ${1:-0 32 64 96}; do
  if [ "$k" = 0 ]; then E=""; else E="SM_CU_CHAIN=$k"; fi
  env $E timeout -k 10 200 $B > $O/c2_$k.log 2>&1 || exit 1
  env $E timeout -k 10 200 $B --disp 256 --emulate-rank 0/8 --shard vd > $O/n8_$k.log 2>&1 || exit 2
done
for f in $O/*.log; do
  python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('%-10s %7.3f ms/frame  latency %7.3f' % ('$(basename $f .log)', d['ms_per_step'], d['latency_ms_per_frame']))"
done
