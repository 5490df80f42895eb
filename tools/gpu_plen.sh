# piece-length sweep: bench + repair statistics per SM_PIECE_LEN
set -o pipefail
mkdir -p gpurun_out
for pl in ${PLS:-256 384 512 768}; do
SM_PIECE_LEN=$pl timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bpl_$pl.log 2>&1 || exit 1
SM_PIECE_LEN=$pl SM_PIECE_DEBUG=1 timeout -k 10 100 python bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/dpl_$pl.log 2>&1 || exit 1
done
