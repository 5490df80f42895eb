# SQ counter passes (wave cycles / waits / instruction mix) over a short bench run, per kernel.
# Usage: bash tools/gpu_sq.sh <tag>   -> gpurun_out/<tag>/sq{1,2}/
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-sq}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $O/sq1 -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu --no-pms --no-segment --no-host-io --inflight 1 > $O/sq1.log 2>&1 || exit 11
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_LEVEL_WAVES SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU -d $O/sq2 -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu --no-pms --no-segment --no-host-io --inflight 1 > $O/sq2.log 2>&1 || exit 12
echo done
