#!/bin/bash
# pgrad tail with the kernel-parameter update from LDS: parity tests, C4 timeline, A/B bench
set -o pipefail
mkdir -p gpurun_out/r3tail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fastgraph.py tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3tail/pytest.log 2>&1 || { tail -30 gpurun_out/r3tail/pytest.log; exit 1; }
tail -1 gpurun_out/r3tail/pytest.log
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib/libgpk_trace.so
GPK_LIB_PATH=$L timeout -k 10 200 python tools/timeline.py --config C4 --steps 5 > gpurun_out/r3tail/c4.txt 2>&1 || exit 1
AB_C2=1 bash tools/gpu/ab_bench.sh
