#!/bin/bash
# Round 3, second session: GPU suite (parity log), smoke, C4/C2 timelines, C4 A/B vs the previous
# build, the driver-shape bench line, rocprofv3 kernel stats + fp64-MFMA passes for C4 and C2.
set -o pipefail
OUT=gpurun_out/r3s2
mkdir -p $OUT
export TMPDIR=/tmp
export GPK_PARITY_LOG=$OUT/parity.jsonl
rm -f $GPK_PARITY_LOG
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
for c in C4 C2; do
  GPK_LIB_PATH=$L/libgpk_trace.so timeout -k 10 200 python tools/timeline.py --config $c --steps 5 > $OUT/timeline_$c.txt 2>&1 || exit 1
done
if [ "${AB:-1}" = 1 ]; then bash tools/gpu/ab_bench.sh || exit 1; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['step1_per_call']['value'], d['large_factors']['step_ms'], d['large_factors']['spd_inverse_ms'])"
B="bench.py --no-cpu-baseline --no-large --steps 200 --warmup 20 --kernel-iters 20 --step1-calls 50"
C2="tools/run_steps.py --config C2 --steps 20"
run() {  # name, rocprof args, command...
  local n=$1; shift; local args=$1; shift
  timeout -k 10 300 rocprofv3 $args -f csv -d $OUT/$n -o $n -- python3 "$@" > $OUT/$n.log 2>&1 || { echo "$n failed"; tail -20 $OUT/$n.log; exit 1; }
}
for cfg in C4 C2; do
  case $cfg in C4) CMD=$B;; C2) CMD=$C2;; esac
  run trace_$cfg "--kernel-trace --stats" $CMD
  run mops_$cfg "--pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" $CMD
  run util_$cfg "--pmc MfmaUtil" $CMD
  f=$(find $OUT/trace_$cfg -name '*kernel_stats.csv' -print -quit); cp "$f" $OUT/${cfg}_kernel_stats.csv
  python3 tools/pmc_mfma.py --trace $OUT/trace_$cfg --mops $OUT/mops_$cfg --util $OUT/util_$cfg --out $OUT/pmc_mfma_$cfg.json --label "$cfg: $CMD" || exit 1
done
rm -rf $OUT/mops_* $OUT/util_* $OUT/trace_*
ls $OUT
