# round 4: SPL = 4 walker chunk sizes after the scratch fix (variant libraries via SM_LIB) -> gpurun_out/r04am
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04am
mkdir -p $O
b() {  # tag, lib
  SM_LIB=$2 timeout -k 10 300 python3 bench.py --disp 256 --no-cpu --no-pms --no-host-io --steps 20 --warmup 3 > $O/d256_$1.log 2>&1 || return 1
  python3 -c "import json;d=json.loads(open('$O/d256_$1.log').read().strip().splitlines()[-1]);k=d['kernels_ms_per_step'];print('$1', round(d['ms_per_step'],3), {x:round(y,3) for x,y in k.items()})"
}
B=stereomatch_amd/libstereomst.so
V=stereomatch_amd/variants
b base $B || exit 1
b dn6 $V/libstereomst_dn6.so || exit 2
b up4 $V/libstereomst_up4.so || exit 3
b dn3 $V/libstereomst_dn3.so || exit 4
b base2 $B || exit 5
for n in dn6 up4 dn3; do
  SM_LIB=$V/libstereomst_$n.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "256" > $O/tests_$n.log 2>&1 || { tail -20 $O/tests_$n.log; exit 6; }
  echo "$n $(tail -1 $O/tests_$n.log)"
done
