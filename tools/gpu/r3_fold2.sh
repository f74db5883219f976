#!/bin/bash
# batch begin/report folded into the step launches: fast-graph, chain and parity GPU tests, then
# the C4 A/B (step1_per_call) against the previous library
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_fastgraph.py tests/test_gpu_chain.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/r3fold2_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r3fold2_pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/r3fold2_pytest.log | head -30; exit 1; fi
bash tools/gpu/ab_bench.sh
