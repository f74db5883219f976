# round 6: C2 chain_multi pass order -- bitwise A/B of loss / grad / trajectory against the
# previous build, then the 1D / chain GPU tests
set -o pipefail
OUT=${OUT:-gpurun_out/r6c2b}
mkdir -p $OUT
export TMPDIR=/tmp
for c in C2 C1; do
  GPK_LIB_PATH=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib/libgpk_base.so timeout -k 10 200 python -u tools/ab_dump.py --config $c --out $OUT/base_$c.npz > /dev/null 2>&1 || exit 1
  timeout -k 10 200 python -u tools/ab_dump.py --config $c --out $OUT/new_$c.npz > /dev/null 2>&1 || exit 1
  python3 -c "
import numpy as np,sys
a=np.load('$OUT/base_$c.npz'); b=np.load('$OUT/new_$c.npz')
print('$c', {k: bool(np.array_equal(a[k], b[k])) for k in a.files})"
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_chain_multi.py tests/test_gpu_parity.py tests/test_gpu_dclass.py tests/test_gpu_accuracy.py \
  > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/tests.log | head -30; exit 1; }
