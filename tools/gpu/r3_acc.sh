#!/bin/bash
# accuracy diagnosis: device K vs oracle K, device gradient vs the long-double yardstick
set -o pipefail
OUT=gpurun_out/r3acc
mkdir -p $OUT
export TMPDIR=/tmp
for c in ${@:-C2 C4}; do
  timeout -k 10 700 python -u tools/gpu_accuracy_diag.py $c > $OUT/diag_$c.json 2> $OUT/diag_$c.err || { echo "diag $c failed"; tail -20 $OUT/diag_$c.err; exit 1; }
  cat $OUT/diag_$c.json
done
