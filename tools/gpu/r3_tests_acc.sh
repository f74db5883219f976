#!/bin/bash
# full GPU suite (with the parity log), then the accuracy diagnosis of the given configs
set -o pipefail
OUT=gpurun_out/r3t
mkdir -p $OUT
export TMPDIR=/tmp
export GPK_PARITY_LOG=$OUT/parity.jsonl
rm -f $GPK_PARITY_LOG
timeout -k 10 700 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" $OUT/pytest.log | head -40; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest aborted rc=$rc"; exit 1; fi
for c in "$@"; do
  timeout -k 10 700 python -u tools/gpu_accuracy_diag.py $c > $OUT/diag_$c.json 2> $OUT/diag_$c.err || { echo "diag $c failed"; tail -20 $OUT/diag_$c.err; exit 1; }
  cat $OUT/diag_$c.json
done
