#!/bin/bash
# round 4 session 3: C5 kernel trace + fp64-MFMA counter passes at the final tree (plain products
# on rocBLAS); outputs under gpurun_out/r4c5
set -o pipefail
OUT=gpurun_out/r4c5
mkdir -p $OUT
export TMPDIR=/tmp
C5="tools/run_steps.py --config C5 --steps 3"
run() {  # name, rocprof args, command...
  local n=$1; shift; local args=$1; shift
  timeout -k 10 300 rocprofv3 $args -f csv -d $OUT/$n -o $n -- python3 "$@" > $OUT/$n.log 2>&1 || { echo "$n failed"; tail -20 $OUT/$n.log; exit 1; }
}
run trace_C5 "--kernel-trace --stats" $C5
run mops_C5 "--pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" $C5
run util_C5 "--pmc MfmaUtil" $C5
f=$(find $OUT/trace_C5 -name '*kernel_stats.csv' -print -quit); cp "$f" $OUT/C5_kernel_stats.csv
python3 tools/pmc_mfma.py --trace $OUT/trace_C5 --mops $OUT/mops_C5 --util $OUT/util_C5 --out $OUT/pmc_mfma_C5.json --label "C5: $C5" || exit 1
rm -rf $OUT/mops_* $OUT/util_*
ls $OUT
