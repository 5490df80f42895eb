# SQ counter passes (wave cycles / waits / instruction mix) per kernel over one frame of a share
# (tools/round_probe.py), one frame at a time.  Usage: bash tools/gpu_sq_share.sh <tag> "<probe args>"
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-sqs}
A=${2:---views 1 --D 64 --d0 0 --dtotal 256}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $O/sq1 -o run --output-format csv -- python tools/round_probe.py $A --frames 1 --warmup 1 > $O/sq1.log 2>&1 || exit 11
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_LEVEL_WAVES SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU -d $O/sq2 -o run --output-format csv -- python tools/round_probe.py $A --frames 1 --warmup 1 > $O/sq2.log 2>&1 || exit 12
python tools/sq_summary.py $O/sq1 $O/sq2 > $O/sq_summary.txt 2>&1
cat $O/sq_summary.txt
echo done
