# round 6: class sums of G_K / G_D in the GEMM epilogues -- tests, then the same-box A/B
set -o pipefail
OUT=${OUT:-gpurun_out/r6cb}
TESTS=${TESTS:-tests/test_gpu_dclass.py tests/test_gpu_parity.py tests/test_gpu_accuracy.py}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS \
  > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/tests.log | head -30; exit 1; }
timeout -k 10 400 python -u tools/ab_flags.py --config C4 --flags 0 4194304 --reps 3 > $OUT/ab.txt 2>&1 || { tail $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
