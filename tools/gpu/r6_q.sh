# round 6: quarter items first in the 128-wide update -- bitwise tests, then the interleaved A/B
set -o pipefail
OUT=${OUT:-gpurun_out/r6q}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py::test_wide_inverse_quarter_tiles_bitwise_whole_tiles \
  "tests/test_gpu_parity.py::test_loss_grad_big_spd_path" tests/test_gpu_timeout.py::test_big_wide_timeout_undoes_batch \
  > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/tests.log | head -30; exit 1; }
timeout -k 10 400 python -u tools/c5_qfirst_ab.py 3 > $OUT/ab.txt 2>&1 || { tail $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
