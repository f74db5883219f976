# round 6: ADVICE regression tests (unequal wide factors, wide gather on every axis, second-chunk
# failure), the C5 inverse pieces with the per-launch flop accounting
set -o pipefail
OUT=${OUT:-gpurun_out/r6a}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_dclass.py tests/test_gpu_timeout.py "tests/test_gpu_parity.py::test_loss_grad_big_spd_path" \
  > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/tests.log | head -30; exit 1; }
timeout -k 10 300 python -u tools/c5_pieces.py > $OUT/c5_pieces.txt 2>&1 || { tail -20 $OUT/c5_pieces.txt; exit 1; }
cat $OUT/c5_pieces.txt
