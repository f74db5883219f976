#!/bin/bash
# C5 large-path refinement modes: accuracy vs the yardstick fixture + step time, then preds probe
set -o pipefail
OUT=gpurun_out/r3ref
mkdir -p $OUT
export TMPDIR=/tmp
for f in 0 8192 16384; do
  timeout -k 10 300 python -u tools/gpu_accuracy_diag.py C5 --quick --flags $f > $OUT/diag_$f.json 2> $OUT/diag_$f.err || { echo "diag $f failed"; tail -20 $OUT/diag_$f.err; exit 1; }
  cat $OUT/diag_$f.json
  timeout -k 10 300 python tools/run_steps.py --config C5 --steps 6 --flags $f > $OUT/steps_$f.txt 2>&1 || { cat $OUT/steps_$f.txt; exit 1; }
  cat $OUT/steps_$f.txt
done
timeout -k 10 400 python -u tools/probe_predict.py 512 4096 > $OUT/probe_predict.txt 2>&1 || { cat $OUT/probe_predict.txt; exit 1; }
cat $OUT/probe_predict.txt
