# round 6: quarter-item loop with 4 K-steps of loads in flight -- bitwise tests, then a same-box A/B
# against the previous commit's library (tools/ab/libgpk_prev.so) and the update timeline
set -o pipefail
OUT=${OUT:-gpurun_out/r6q2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py::test_wide_inverse_quarter_tiles_bitwise_whole_tiles \
  "tests/test_gpu_parity.py::test_loss_grad_big_spd_path" > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/tests.log | head -30; exit 1; }
for r in 0 1; do
  GPK_LIB_PATH=$PWD/tools/ab/libgpk_prev.so timeout -k 10 300 python -u tools/c5_qfirst_ab.py 1 > $OUT/ab_prev_$r.txt 2>&1 || { tail $OUT/ab_prev_$r.txt; exit 1; }
  sed 's/^/prev /' $OUT/ab_prev_$r.txt
  timeout -k 10 300 python -u tools/c5_qfirst_ab.py 1 > $OUT/ab_new_$r.txt 2>&1 || { tail $OUT/ab_new_$r.txt; exit 1; }
  sed 's/^/new  /' $OUT/ab_new_$r.txt
done
GPK_LIB_PATH=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib/libgpk_trace.so timeout -k 10 200 python -u tools/big_timeline.py --reps 3 > $OUT/tl.txt 2>&1 || { tail $OUT/tl.txt; exit 1; }
cat $OUT/tl.txt
