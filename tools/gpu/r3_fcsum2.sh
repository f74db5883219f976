#!/bin/bash
# fused class sums (LDS-bin form too): tests, C4 / C2 ms/step default vs GPK_FLAG_NO_FUSED_CSUM
set -o pipefail
mkdir -p gpurun_out/fcs2
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_dclass.py tests/test_gpu_parity.py tests/test_gpu_fastgraph.py tests/test_gpu_fullsize.py tests/test_gpu_chain_multi.py -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/fcs2/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/fcs2/pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/fcs2/pytest.log | head -30; exit 1; fi
for rep in 1 2 3; do
  for fl in 0 65536; do
    timeout -k 10 200 python tools/run_steps.py --config C4 --steps 500 --flags $fl > gpurun_out/fcs2/s.txt 2>&1 || { cat gpurun_out/fcs2/s.txt; exit 1; }
    head -1 gpurun_out/fcs2/s.txt
    timeout -k 10 200 python tools/run_steps.py --config C2 --steps 100 --flags $fl > gpurun_out/fcs2/s.txt 2>&1 || { cat gpurun_out/fcs2/s.txt; exit 1; }
    head -1 gpurun_out/fcs2/s.txt
  done
done
GPK_LIB_PATH=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib/libgpk_trace.so timeout -k 10 200 python tools/timeline.py --config C4 --steps 5 > gpurun_out/fcs2/tl.txt 2>&1
grep -E "gemm stage 10|class_sum|pg |pgrad|fin:" gpurun_out/fcs2/tl.txt
