# round 4: GPU schedule forest (checked against the host build), the segment min-size pair dedupe, the
# PMS suite, the 100-call C2 frame (GPU vs host forest), chain threshold sweep, segment latency -> gpurun_out/r04n
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_pms_gpu.py \
  -k "gpu_forest_matches" > $O/tests_forest.log 2>&1 || { tail -40 $O/tests_forest.log; exit 1; }
tail -3 $O/tests_forest.log
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "segment" > $O/tests_seg.log 2>&1 || { tail -40 $O/tests_seg.log; exit 1; }
tail -3 $O/tests_seg.log
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/test_pms_gpu.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 2 > $O/pms100.log 2>&1 || exit 2
tail -1 $O/pms100.log | cut -c1-1500
SM_PMS_HOST_FOREST=1 timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 2 > $O/pms100_hostforest.log 2>&1 || exit 3
echo "host forest: $(tail -1 $O/pms100_hostforest.log | cut -c1-420)"
SM_PMS_CHAIN_STREAM=1 timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 2 > $O/pms100_onestream.log 2>&1 || exit 3
echo "chain stream: $(tail -1 $O/pms100_onestream.log | cut -c1-420)"
for cm in 48 192; do
  SM_PMS_CHAIN_MIN=$cm timeout -k 10 300 python3 tools/pms_bench.py 1920 1200 128 100 --reps 2 > $O/pms100_cm$cm.log 2>&1 || exit 4
  echo "chain_min $cm: $(tail -1 $O/pms100_cm$cm.log | cut -c1-420)"
done
SM_SEG_DEBUG=1 timeout -k 10 300 python bench.py --segment-c 5000 --no-cpu --no-pms --steps 16 --warmup 4 --inflight 0 > $O/seg_0.log 2> $O/seg_0.err || exit 5
grep segment_gpu $O/seg_0.err | tail -3
python3 -c "import json;d=json.loads(open('$O/seg_0.log').read().strip().splitlines()[-1]);print('seg inflight 0', round(d['ms_per_step'],3), 'latency', d.get('latency_ms_per_frame'), {k: round(v,2) for k,v in d['stages_ms'].items()})"
SM_SEG_NODEDUP=1 SM_SEG_DEBUG=1 timeout -k 10 300 python bench.py --segment-c 5000 --no-cpu --no-pms --steps 16 --warmup 4 --inflight 0 > $O/seg_0_nodedup.log 2> $O/seg_0_nodedup.err || exit 6
grep segment_gpu $O/seg_0_nodedup.err | tail -2
python3 -c "import json;d=json.loads(open('$O/seg_0_nodedup.log').read().strip().splitlines()[-1]);print('seg nodedup inflight 0', round(d['ms_per_step'],3), 'latency', d.get('latency_ms_per_frame'))"
for fl in 0 3; do
  SM_SEG_FLATTEN=$fl SM_SEG_DEBUG=1 timeout -k 10 300 python bench.py --segment-c 5000 --no-cpu --no-pms --steps 16 --warmup 4 --inflight 0 > $O/seg_0_fl$fl.log 2> $O/seg_0_fl$fl.err || exit 7
  grep segment_gpu $O/seg_0_fl$fl.err | tail -1
  python3 -c "import json;d=json.loads(open('$O/seg_0_fl$fl.log').read().strip().splitlines()[-1]);print('seg flatten $fl inflight 0', round(d['ms_per_step'],3), 'latency', d.get('latency_ms_per_frame'))"
done
