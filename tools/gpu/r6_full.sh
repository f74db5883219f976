# round 6: the whole GPU suite (parity log), smoke, a C5 trajectory check
set -o pipefail
OUT=${OUT:-gpurun_out/r6full}
mkdir -p $OUT
export TMPDIR=/tmp GPK_PARITY_LOG=$PWD/$OUT/parity.jsonl
rm -f $GPK_PARITY_LOG
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
grep -E "FAILED|^E " $OUT/pytest.log | head -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u tools/c5_traj_check.py > $OUT/traj.txt 2>&1 || { tail $OUT/traj.txt; exit 1; }
cat $OUT/traj.txt
exit $rc
