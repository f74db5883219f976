# round 6: the Adam block forms pg from the group partials in its own load batch -- bitwise
# A/B of loss / grad / trajectory against the previous build, the class-pipe tests, then the
# same-box speed A/B at C4
set -o pipefail
OUT=${OUT:-gpurun_out/r6pgd}
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
mkdir -p $OUT
export TMPDIR=/tmp
for c in C4 C2 C5; do
  GPK_LIB_PATH=$L/libgpk_base.so timeout -k 10 200 python -u tools/ab_dump.py --config $c --out $OUT/base_$c.npz > /dev/null 2>&1 || exit 1
  timeout -k 10 200 python -u tools/ab_dump.py --config $c --out $OUT/new_$c.npz > /dev/null 2>&1 || exit 1
  python3 -c "
import numpy as np
a=np.load('$OUT/base_$c.npz'); b=np.load('$OUT/new_$c.npz')
print('$c', {k: bool(np.array_equal(a[k], b[k])) for k in a.files})"
  rm -f $OUT/base_$c.npz $OUT/new_$c.npz  # (C5's dumps alone exceed gpurun_out's 64 MiB)
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_cls_pipe.py \
  > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/tests.log | head -30; exit 1; }
timeout -k 10 500 python -u tools/ab_libs.py --config C4 --libs $L/libgpk_base.so $L/libgpk.so --reps 3 > $OUT/ab_c4.txt 2>&1 || { tail $OUT/ab_c4.txt; exit 1; }
cat $OUT/ab_c4.txt
