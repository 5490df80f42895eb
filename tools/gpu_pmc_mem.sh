# Memory-pipeline PMC passes (TA busy / stalls, L1 pending stalls and L2 request latency, L2
# hits) over one-frame-at-a-time bench runs; per-kernel sums via tools/sq_summary.py.
# Usage (on the box): bash tools/gpu_pmc_mem.sh <tag>   -> gpurun_out/<tag>/m{1,2}/
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-mem}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
B="python bench.py --steps 1 --warmup 1 --no-cpu --no-host-io --inflight 1"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES -d $O/m1 -o run --output-format csv -- $B > $O/m1.log 2>&1 || exit 11
timeout -k 10 120 rocprofv3 --pmc TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ_LAT TCP_TCC_READ_REQ TCP_READ_TAGCONFLICT_STALL_CYCLES TCC_HIT TCC_MISS TA_DATA_STALLED_BY_TC_CYCLES -d $O/m2 -o run --output-format csv -- $B > $O/m2.log 2>&1 || exit 12
python tools/sq_summary.py $O/m1 $O/m2
