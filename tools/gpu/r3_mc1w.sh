#!/bin/bash
# chain_multi with the one-wave pivot (16 VGPRs spilled): chain tests, C2 A/B vs the previous build
set -o pipefail
mkdir -p gpurun_out/mc1w
export TMPDIR=/tmp
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain_multi.py tests/test_gpu_chain.py -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/mc1w/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/mc1w/pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/mc1w/pytest.log | head -30; exit 1; fi
for rep in 1 2 3; do
  for lib in libgpk.so libgpk_ab.so; do
    GPK_LIB_PATH=$L/$lib timeout -k 10 200 python tools/run_steps.py --config C2 --steps 100 > gpurun_out/mc1w/steps.txt 2>&1 || { cat gpurun_out/mc1w/steps.txt; exit 1; }
    echo "$lib $(head -1 gpurun_out/mc1w/steps.txt)"
  done
done
