# round 6: pipelined class values (next step's class values in the pgrad launch) -- bitwise
# tests against GPK_FLAG_NO_CLASS_PIPE, then the same-box A/B at C4 and C2
set -o pipefail
OUT=${OUT:-gpurun_out/r6pipe}
TESTS=${TESTS:-tests/test_gpu_cls_pipe.py}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu $TESTS \
  > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/tests.log | head -30; exit 1; }
timeout -k 10 400 python -u tools/ab_flags.py --config C4 --flags 0 8388608 --reps 3 > $OUT/ab_c4.txt 2>&1 || { tail $OUT/ab_c4.txt; exit 1; }
cat $OUT/ab_c4.txt
timeout -k 10 300 python -u tools/ab_flags.py --config C2 --flags 0 8388608 --reps 2 > $OUT/ab_c2.txt 2>&1 || { tail $OUT/ab_c2.txt; exit 1; }
cat $OUT/ab_c2.txt
