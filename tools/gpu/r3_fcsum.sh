#!/bin/bash
# class sums fused into the contraction launch: tests, C4 A/B vs the previous build
set -o pipefail
mkdir -p gpurun_out/fcs
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_dclass.py tests/test_gpu_parity.py tests/test_gpu_fastgraph.py tests/test_gpu_fullsize.py tests/test_gpu_accuracy.py tests/test_gpu_golden.py -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/fcs/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/fcs/pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/fcs/pytest.log | head -30; exit 1; fi
bash tools/gpu/ab_bench.sh
