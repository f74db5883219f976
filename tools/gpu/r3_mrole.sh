#!/bin/bash
# chain_multi with the diagonal tiles spread over the macro row: tests, C2 timeline, A/B (C2 + C4)
set -o pipefail
mkdir -p gpurun_out/r3mrole
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_chain_multi.py tests/test_gpu_parity.py tests/test_gpu_accuracy.py tests/test_gpu_golden.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3mrole/pytest.log 2>&1 || { tail -30 gpurun_out/r3mrole/pytest.log; exit 1; }
tail -1 gpurun_out/r3mrole/pytest.log
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib/libgpk_trace.so
GPK_LIB_PATH=$L timeout -k 10 200 python tools/timeline.py --config C2 --steps 5 > gpurun_out/r3mrole/c2.txt 2>&1 || exit 1
AB_C2=1 bash tools/gpu/ab_bench.sh
