# round 6: kernel durations of C4 with the epilogue class sums (flags 0) and the class-sum launch
set -o pipefail
OUT=${OUT:-gpurun_out/r6cbp}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for f in 0 4194304; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/f$f -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/run_steps.py --config C4 --steps 300 --flags $f > $GRAFT_REPO_ROOT/$OUT/f$f.log 2>&1 || exit 1
done
cd $GRAFT_REPO_ROOT
python3 tools/kernel_db_stats.py $OUT/f0 $OUT/f4194304
