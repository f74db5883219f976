#!/bin/bash
# Iteration loop on one GPU box: selected GPU tests (default: all), a short bench line, and a
# rocprofv3 kernel trace + stats of the bench.   usage: tools/gpu_quick.sh [pytest selector...]
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
SEL=${@:-tests}
timeout -k 10 600 python -u -m pytest $SEL -q -m gpu -x --timeout 120 --timeout-method thread > $OUT/quick_pytest.log 2>&1; rc=$?
tail -3 $OUT/quick_pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" $OUT/quick_pytest.log | head -30; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest aborted rc=$rc"; exit 1; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --no-large --steps 300 > $OUT/quick_bench.json 2> $OUT/quick_bench.err || { echo bench failed; tail -20 $OUT/quick_bench.err; exit 1; }
cat $OUT/quick_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/quick_prof -o q -- python3 bench.py --no-cpu-baseline --no-large --steps 100 > $OUT/quick_prof.log 2>&1 || { echo rocprof failed; tail -20 $OUT/quick_prof.log; exit 1; }
python3 tools/trace_summary.py $OUT/quick_prof
