#!/bin/bash
# C2 with class-operand GEMVs (no Kc / D matrices written by the inverse): 1D GPU tests, then
# ms/step default vs GPK_FLAG_MATRIX_GEMV (32768), interleaved, same library
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain_multi.py tests/test_gpu_accuracy.py tests/test_gpu_parity.py tests/test_gpu_fastgraph.py tests/test_gpu_dropin.py -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/r3cg_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r3cg_pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/r3cg_pytest.log | head -30; exit 1; fi
for rep in 1 2 3; do
  for fl in 0 32768; do
    timeout -k 10 200 python tools/run_steps.py --config C2 --steps 100 --flags $fl > gpurun_out/r3cg_steps.txt 2>&1 || { cat gpurun_out/r3cg_steps.txt; exit 1; }
    head -1 gpurun_out/r3cg_steps.txt
  done
done
tail -1 gpurun_out/r3cg_steps.txt
