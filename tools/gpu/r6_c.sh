# round 6: the two round-5-loosened tests, now gated against yardsticks (T3072 fixture; the DD
# contraction's own error on identical G)
set -o pipefail
OUT=${OUT:-gpurun_out/r6c}
mkdir -p $OUT
export TMPDIR=/tmp GPK_PARITY_LOG=$PWD/$OUT/parity.jsonl
rm -f $GPK_PARITY_LOG
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py::test_tile128_and_64x64_stages_vs_yardstick \
  tests/test_gpu_accuracy.py::test_dd_contraction_against_yardstick > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
cat $GPK_PARITY_LOG 2>/dev/null | tail -8
[ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/tests.log | head -30; exit 1; }
