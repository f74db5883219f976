# round 6: large advection factors refine A's forward solve alone -- C5 parity tests, plan tests,
# a 20-step trajectory against REFINE_ALL, the C5 step
set -o pipefail
OUT=${OUT:-gpurun_out/r6f}
mkdir -p $OUT
export TMPDIR=/tmp GPK_PARITY_LOG=$PWD/$OUT/parity.jsonl
rm -f $GPK_PARITY_LOG
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \

  tests/test_gpu_fullsize.py > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/tests.log | head -30; exit 1; }
grep C5 $GPK_PARITY_LOG | head -3
timeout -k 10 300 python -u tools/c5_traj_check.py > $OUT/traj.txt 2>&1 || { tail $OUT/traj.txt; exit 1; }
cat $OUT/traj.txt
