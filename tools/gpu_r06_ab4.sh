# round 6 A/B 4: the up chain on 4-byte image records -- parity, timing against the 8-byte variant, PMC traffic
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ab4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 2; }
tail -1 $O/tests.log
E="--emulate-rank 0/8 --frame-groups 1"
V=SM_LIB=variants/rec8/libstereomst.so
BASE_ARGS="--steps 20 --warmup 5 --no-cpu --no-host-io --no-pms --no-segment" bash tools/gpu_ab.sh \
  "c2||" "c2_rec8|$V|" "share||$E" "share_rec8|$V|$E" "c2_b||" "c2_rec8_b|$V|" "d||$E --shard d" "d_rec8|$V|$E --shard d" || exit 3
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu --no-host-io --no-pms --no-segment --inflight 1 > $O/pmc_fetch.log 2>&1 || exit 13
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu --no-host-io --no-pms --no-segment --inflight 1 > $O/pmc_write.log 2>&1 || exit 14
python tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write auto $O/pmc_traffic.json > $O/pmc_traffic.log 2>&1 || exit 15
python3 -c "import json;d=json.load(open('$O/pmc_traffic.json'));print({k:round(v['hbm_bytes_per_frame']/1e9,3) for k,v in d.items() if isinstance(v,dict)})"
echo done
