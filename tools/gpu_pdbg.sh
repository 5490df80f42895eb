set -o pipefail
mkdir -p gpurun_out
for pl in 512 256; do
SM_PIECE_LEN=$pl SM_PIECE_DEBUG=2 timeout -k 10 120 python bench.py --dev --steps 1 --warmup 1 --no-cpu > gpurun_out/pdbg_$pl.log 2>&1 || exit 1
done
