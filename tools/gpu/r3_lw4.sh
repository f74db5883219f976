#!/bin/bash
# chain_kernel with L_k^{-1} as self-validating words: full GPU suite, C4 timeline, C4 A/B vs the previous build
set -o pipefail
mkdir -p gpurun_out/r3lw4
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3lw4/pytest.log 2>&1 || { tail -30 gpurun_out/r3lw4/pytest.log; exit 1; }
tail -1 gpurun_out/r3lw4/pytest.log
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
GPK_LIB_PATH=$L/libgpk_trace.so timeout -k 10 200 python tools/timeline.py --config C4 --steps 5 > gpurun_out/r3lw4/c4.txt 2>&1 || exit 1
bash tools/gpu/ab_bench.sh
