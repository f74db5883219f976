#!/bin/bash
# C2 (1D N = 2048): GPU tests of the 1D path, then ms/step with libgpk.so vs libgpk_ab.so (interleaved)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_chain_multi.py tests/test_gpu_accuracy.py tests/test_gpu_parity.py -q -m gpu -x --timeout 300 --timeout-method thread -k "C2 or c2 or 1d or multi" > gpurun_out/r3c2_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r3c2_pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/r3c2_pytest.log | head -30; exit 1; fi
L=gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
for rep in 1 2 3; do
  for lib in libgpk.so libgpk_ab.so; do
    GPK_LIB_PATH=$PWD/$L/$lib timeout -k 10 200 python tools/run_steps.py --config C2 --steps 100 > gpurun_out/r3c2_steps.txt 2>&1 || { cat gpurun_out/r3c2_steps.txt; exit 1; }
    echo "$lib $(head -1 gpurun_out/r3c2_steps.txt)"
  done
done
tail -1 gpurun_out/r3c2_steps.txt
