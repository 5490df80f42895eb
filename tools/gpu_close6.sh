# Close of round 6 on one GPU box.  Outputs under gpurun_out/<tag>/ (copied to profiles/r06/ afterwards):
#  * layout invariants (no filter), smoke(), the full -m gpu suite, the degenerate-tree file;
#  * the build's sha256 (every summary below is of this library);
#  * MST-only kernel summaries (--no-pms --no-segment): frames in flight and one frame at a time, the
#    latter's k_up_walk average against the same run's roofline.isolated.avg_launch_ms;
#  * FETCH_SIZE / WRITE_SIZE passes -> profiles/pmc_traffic.json, then the driver's command line;
#  * the 100-call MST_PMS frame, C4 on one GPU, the N = 8 per-rank emulations, the C3 pair line,
#    guided, and the context memory at C2 / C3.
# Usage (on the box): bash tools/gpu_close6.sh r06close [skip-tests]
set -o pipefail
TAG=${1:-r06close}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
sha256sum stereomatch_amd/libstereomst.so | cut -c1-16 > $O/build_sha.txt
echo "build sha256:$(cat $O/build_sha.txt)"
timeout -k 10 300 python tools/layout_check.py > $O/layout_check.log 2>&1 || { cat $O/layout_check.log; exit 1; }
if [ "$2" != "skip-tests" ]; then
  bash tools/gpu_tests.sh $TAG || exit 2
fi
M="--no-cpu --no-host-io --no-pms --no-segment"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python bench.py --steps 10 --warmup 2 $M > $O/stats_bench.log 2>&1 || exit 11
python tools/timed_region.py $O/stats/run_kernel_trace.csv $O/stats_bench.log > $O/timed_region.txt 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats1 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 $M --inflight 1 > $O/stats1_bench.log 2>&1 || exit 13
python3 - $O <<'EOF' > $O/isolated_check.txt || exit 14
import csv, json, sys
o = sys.argv[1]
line = json.loads([l for l in open(o + "/stats1_bench.log") if l.startswith('{"metric')][-1])
iso = line["roofline"]["isolated"]["avg_launch_ms"] * 1e3
rows = [r for r in csv.DictReader(open(o + "/stats1/run_kernel_stats.csv")) if r["Name"].startswith("void k_up_walk<")]
calls = sum(int(r["Calls"]) for r in rows)
avg = sum(float(r["TotalDurationNs"]) for r in rows) / calls / 1e3
print("build sha256:%s" % open(o + "/build_sha.txt").read().strip())
print("k_up_walk one frame at a time (rocprofv3 --stats, %d launches): avg %.1f us" % (calls, avg))
print("same run's roofline.isolated.avg_launch_ms (HIP events): %.1f us -> ratio %.3f" % (iso, avg / iso))
EOF
cat $O/isolated_check.txt
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python bench.py --steps 2 --warmup 1 $M --inflight 1 > $O/pmc_fetch.log 2>&1 || exit 15
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python bench.py --steps 2 --warmup 1 $M --inflight 1 > $O/pmc_write.log 2>&1 || exit 16
python tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write auto $O/pmc_traffic.json > $O/pmc_traffic.log 2>&1 || exit 17
cp $O/pmc_traffic.json profiles/pmc_traffic.json  # the lines below report this traffic (same_build)
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.log 2>&1 || exit 18
python3 -c "import json;d=json.loads(open('$O/bench_default.log').read().strip().splitlines()[-1]);print('driver line', round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],3), 'same_build', d['roofline'].get('traffic_source',{}).get('same_build'), 'pms frame', round(d.get('pms',{}).get('frame_s',0),3))" || true
timeout -k 10 300 python tools/pms_bench.py 1920 1200 128 100 --reps 2 > $O/pms100.log 2>&1 || exit 19
tail -1 $O/pms100.log | cut -c1-300
timeout -k 10 300 python bench.py --disp 256 --steps 20 --warmup 5 $M > $O/c4_1gpu.log 2>&1 || exit 20
for spec in "0/8 --frame-groups 1" "0/8 --frame-groups 2" "0/8 --shard d --frame-groups 1"; do
  set -- $spec
  tagn=$(echo "$spec" | tr ' /' '__' | tr -d '-')
  timeout -k 10 300 python bench.py --emulate-rank $spec --steps 20 --warmup 5 $M > $O/emu_$tagn.log 2>&1 || exit 21
done
timeout -k 10 400 python bench.py --mode batch --steps 10 --warmup 3 $M > $O/c3_batch.log 2>&1 || exit 22
timeout -k 10 300 python bench.py --aggregator guided --steps 20 --warmup 5 $M > $O/guided.log 2>&1 || exit 23
timeout -k 10 300 python tools/mem_probe.py 3840 2160 256 > $O/mem_c3.log 2>&1 || exit 24
timeout -k 10 300 python tools/mem_probe.py 1920 1200 128 > $O/mem_c2.log 2>&1 || exit 25
for f in c4_1gpu emu_0_8_framegroups_1 emu_0_8_framegroups_2 emu_0_8_shard_d_framegroups_1 c3_batch guided; do
  python3 -c "import json;d=json.loads(open('$O/$f.log').read().strip().splitlines()[-1]);print('$f', round(d['ms_per_step'],3), d['config'].get('workload'), 'inflight', d.get('frames_in_flight'))" || true
done
grep -h context $O/mem_c3.log $O/mem_c2.log
echo done
