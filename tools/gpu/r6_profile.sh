#!/bin/bash
# Round-6 measurement session: GPU suite (parity log), smoke, the driver-shape bench line, and
# rocprofv3 traces + PMC passes (HBM FETCH/WRITE, fp64 MFMA) for C4 (bench), C5 and C2.
set -o pipefail
OUT=${OUT:-gpurun_out/r6p}
TREE=$(cat tools/gpu/TREE.txt 2>/dev/null)
mkdir -p $OUT
export TMPDIR=/tmp
export GPK_PARITY_LOG=$OUT/parity.jsonl
rm -f $GPK_PARITY_LOG
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 700 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
  tail -3 $OUT/pytest.log
  if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" $OUT/pytest.log | head -40; fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest aborted rc=$rc"; exit 1; fi
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; cat $OUT/smoke.log; exit 1; }
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
ldd gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib/libgpk.so > $OUT/ldd.txt
B="bench.py --no-cpu-baseline --no-large --steps 200 --warmup 20 --kernel-iters 20 --step1-calls 50"
C5="tools/run_steps.py --config C5 --steps 3"
C2="tools/run_steps.py --config C2 --steps 20"
run() {  # name, rocprof args, command...
  local n=$1; shift; local args=$1; shift
  timeout -k 10 300 rocprofv3 $args -f csv -d $OUT/$n -o $n -- python3 "$@" > $OUT/$n.log 2>&1 || { echo "$n failed"; tail -20 $OUT/$n.log; exit 1; }
}
for cfg in ${CFGS:-C4 C5 C2}; do
  case $cfg in C4) CMD=$B;; C5) CMD=$C5;; C2) CMD=$C2;; esac
  run trace_$cfg "--kernel-trace --stats" $CMD
  run mops_$cfg "--pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" $CMD
  run util_$cfg "--pmc MfmaUtil" $CMD
  f=$(find $OUT/trace_$cfg -name '*kernel_stats.csv' -print -quit); cp "$f" $OUT/${cfg}_kernel_stats.csv
  python3 tools/pmc_mfma.py --trace $OUT/trace_$cfg --mops $OUT/mops_$cfg --util $OUT/util_$cfg --out $OUT/pmc_mfma_$cfg.json --label "$cfg: $CMD" || exit 1
done
for cfg in ${HBM_CFGS:-C4 C5}; do
  case $cfg in C4) CMD=$B;; C5) CMD=$C5;; C2) CMD=$C2;; esac
  run fetch_$cfg "--pmc FETCH_SIZE" $CMD
  run write_$cfg "--pmc WRITE_SIZE" $CMD
  python3 tools/pmc_summary.py $OUT/fetch_$cfg $OUT/write_$cfg $OUT/pmc_${cfg,,}.json "$TREE" > /dev/null || exit 1
done
rm -rf $OUT/mops_* $OUT/util_* $OUT/fetch_* $OUT/write_*
ls $OUT
