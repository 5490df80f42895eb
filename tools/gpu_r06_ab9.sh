# round 6 A/B 9: kernel traces of the default in-flight C2 bench, committed build vs compact rows, interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ab9
mkdir -p $O
P="--dev --steps 20 --warmup 5 --no-cpu --no-host-io --no-pms --no-segment"
for r in 1 2; do
  SM_LIB=variants/head/libstereomst.so timeout -k 10 300 rocprofv3 --kernel-trace -d $O/head_$r -o run -- python bench.py $P > $O/head_$r.log 2>&1 || exit 4
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/new_$r -o run -- python bench.py $P > $O/new_$r.log 2>&1 || exit 5
done
echo done
