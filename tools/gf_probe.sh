cd /tmp && export TMPDIR=/tmp
for d in 0 4 6; do
  SM_GF_DBG=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/probe_$d -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-pms --no-host-io --aggregator guided --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/probe_$d.log 2>&1 || exit 1
done
