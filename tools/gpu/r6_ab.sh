# round 6: GPU tests named by TESTS, then a same-box A/B of gpk/_lib/libgpk.so against
# gpk/_lib/libgpk_base.so (the previous commit's build) on C4
set -o pipefail
OUT=${OUT:-gpurun_out/r6ab}
TESTS=${TESTS:-tests/test_gpu_dclass.py}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS \
  > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/tests.log | head -30; exit 1; }
timeout -k 10 600 python -u tools/ab_libs.py --config ${CONFIG:-C4} --reps ${REPS:-3} \
  --libs gpk/_lib/libgpk_base.so gpk/_lib/libgpk.so > $OUT/ab.txt 2>&1 || { tail $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
