#!/bin/bash
# quarter-tile last round of the 128-wide SPD update: C5 bitwise vs the previous build, the C5
# tests, and the inverse pieces (new, old)
set -o pipefail
mkdir -p gpurun_out/quarter
export TMPDIR=/tmp
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
timeout -k 10 200 python tools/ab_dump.py --config C5 --out /tmp/q_new.npz &&
GPK_LIB_PATH=$L/libgpk_ab.so timeout -k 10 200 python tools/ab_dump.py --config C5 --out /tmp/q_old.npz &&
python3 -c "
import numpy as np
a, b = np.load('/tmp/q_new.npz'), np.load('/tmp/q_old.npz')
print('C5 bitwise new == old:', {k: bool(np.array_equal(a[k], b[k])) for k in a.files})
" || exit 1
timeout -k 10 200 python tools/c5_pieces.py > gpurun_out/quarter/pieces_new.txt 2>&1 && cat gpurun_out/quarter/pieces_new.txt &&
GPK_LIB_PATH=$L/libgpk_ab.so timeout -k 10 200 python tools/c5_pieces.py > gpurun_out/quarter/pieces_old.txt 2>&1 && echo "old:" && cat gpurun_out/quarter/pieces_old.txt || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_accuracy.py -q -m gpu -x --timeout 300 --timeout-method thread -k "C5 or c5 or advection or big" > gpurun_out/quarter/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/quarter/pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/quarter/pytest.log | head -30; exit 1; fi
