#!/bin/bash
# batched class-operand GEMV: 1D tests, C2 default vs GPK_FLAG_MATRIX_GEMV, kernel stats
set -o pipefail
mkdir -p gpurun_out/cg2
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain_multi.py tests/test_gpu_parity.py -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/cg2/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/cg2/pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/cg2/pytest.log | head -30; exit 1; fi
for rep in 1 2 3; do
  for fl in 0 32768; do
    timeout -k 10 200 python tools/run_steps.py --config C2 --steps 100 --flags $fl > gpurun_out/cg2/steps.txt 2>&1 || { cat gpurun_out/cg2/steps.txt; exit 1; }
    head -1 gpurun_out/cg2/steps.txt
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/cg2/prof -o run -- python3 tools/run_steps.py --config C2 --steps 30 > gpurun_out/cg2/prof.log 2>&1 || { tail gpurun_out/cg2/prof.log; exit 1; }
f=$(find gpurun_out/cg2/prof -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv, sys
for r in csv.DictReader(open(sys.argv[1])): print(f\"{r['Name'][:64]:64s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.2f} us\")
" "$f"
