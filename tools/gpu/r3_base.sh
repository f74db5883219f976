#!/bin/bash
# Round-3 baseline on a fresh box: counter list, full GPU suite, bench line, C2/C5 step rates.
set -o pipefail
OUT=gpurun_out/r3base
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || echo "counter list rc=$?"
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" $OUT/pytest.log | head -30; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest aborted rc=$rc"; exit 1; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
for c in C2 C5; do timeout -k 10 200 python tools/run_steps.py --config $c --steps 10 > $OUT/$c.txt 2>&1 || { cat $OUT/$c.txt; exit 1; }; cat $OUT/$c.txt; done
