#!/bin/bash
# gemm_small XCD-aware tile order + nontemporal output stores: parity tests, then the C4 A/B
# (libgpk.so = both, libgpk_x.so = tile order only, libgpk_ab.so = before)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fastgraph.py tests/test_gpu_fullsize.py tests/test_gpu_edges.py -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/r3gx_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r3gx_pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/r3gx_pytest.log | head -30; exit 1; fi
LIBS="libgpk.so libgpk_x.so libgpk_ab.so" bash tools/gpu/ab_bench.sh
