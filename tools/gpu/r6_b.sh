# round 6: the sharded step's 3-collective plan (augmented chain on sharded handles, one
# all-reduce), its tests, the timeout tests and smoke
set -o pipefail
OUT=${OUT:-gpurun_out/r6b}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_shard.py tests/test_gpu_timeout.py > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/tests.log | head -30; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
