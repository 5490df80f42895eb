# round 6: compact A rows -- smoke, the -m gpu suite (degenerate trees last), context memory, C2 / C3 lines
set -o pipefail
TAG=${1:-r06cmp}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_tests.sh $TAG || exit 1
timeout -k 10 300 python tools/mem_probe.py 3840 2160 256 > $O/mem_c3.log 2>&1 || exit 4
timeout -k 10 300 python tools/mem_probe.py 1920 1200 128 > $O/mem_c2.log 2>&1 || exit 5
cat $O/mem_c3.log $O/mem_c2.log | grep context
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-host-io --no-pms --no-segment > $O/c2.log 2>&1 || exit 6
timeout -k 10 400 python bench.py --mode batch --steps 10 --warmup 3 --no-cpu --no-host-io --no-pms --no-segment > $O/c3.log 2>&1 || exit 7
for f in c2 c3; do python3 -c "import json;d=json.loads(open('$O/$f.log').read().strip().splitlines()[-1]);print('$f', round(d['ms_per_step'],3), 'inflight', d['frames_in_flight'], {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})"; done
echo done
