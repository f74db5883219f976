# round 6: a candidate build (libgpk_new.so) against the current one (libgpk.so) -- bitwise A/B of
# loss / grad / trajectory at C4, C2, C5, the class-pipe tests on the candidate, speed A/B at C4
set -o pipefail
OUT=${OUT:-gpurun_out/r6fe}
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
mkdir -p $OUT
export TMPDIR=/tmp
for c in C4 C2 C5; do
  timeout -k 10 200 python -u tools/ab_dump.py --config $c --out $OUT/base_$c.npz > /dev/null 2>&1 || exit 1
  GPK_LIB_PATH=$L/libgpk_new.so timeout -k 10 200 python -u tools/ab_dump.py --config $c --out $OUT/new_$c.npz > /dev/null 2>&1 || exit 1
  python3 -c "
import numpy as np
a=np.load('$OUT/base_$c.npz'); b=np.load('$OUT/new_$c.npz')
print('$c', {k: bool(np.array_equal(a[k], b[k])) for k in a.files})"
  rm -f $OUT/base_$c.npz $OUT/new_$c.npz
done
GPK_LIB_PATH=$L/libgpk_new.so timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_cls_pipe.py \
  > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/tests.log | head -30; exit 1; }
timeout -k 10 500 python -u tools/ab_libs.py --config C4 --libs $L/libgpk.so $L/libgpk_new.so --reps 3 > $OUT/ab_c4.txt 2>&1 || { tail $OUT/ab_c4.txt; exit 1; }
cat $OUT/ab_c4.txt
