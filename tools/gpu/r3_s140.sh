#!/bin/bash
# huge-GEMM LDS stride 140: large-path tests, C5 bitwise vs the previous build, pieces
set -o pipefail
mkdir -p gpurun_out/s140
export TMPDIR=/tmp
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
timeout -k 10 200 python tools/ab_dump.py --config C5 --out /tmp/s_new.npz &&
GPK_LIB_PATH=$L/libgpk_ab.so timeout -k 10 200 python tools/ab_dump.py --config C5 --out /tmp/s_old.npz &&
python3 -c "
import numpy as np
a, b = np.load('/tmp/s_new.npz'), np.load('/tmp/s_old.npz')
print('C5 bitwise new == old:', {k: bool(np.array_equal(a[k], b[k])) for k in a.files})
" || exit 1
timeout -k 10 200 python tools/c5_pieces.py || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_accuracy.py tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_shard.py -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/s140/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/s140/pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/s140/pytest.log | head -30; exit 1; fi
