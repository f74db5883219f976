# round 6: the 128-wide update launch's device timeline (probe build), quarter items first / last
set -o pipefail
OUT=${OUT:-gpurun_out/r6tl}
mkdir -p $OUT
export TMPDIR=/tmp GPK_LIB_PATH=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib/libgpk_trace.so
for f in 0 GPK_FLAG_NO_QUARTER_FIRST; do
  timeout -k 10 200 python -u tools/big_timeline.py --reps 3 --flags $f > $OUT/tl_$f.txt 2>&1 || { tail $OUT/tl_$f.txt; exit 1; }
  cat $OUT/tl_$f.txt
done
