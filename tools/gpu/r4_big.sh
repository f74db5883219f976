#!/bin/bash
# round 4: the large-factor inverse: big-path tests, the pieces' timings, the update launch's
# device timeline (probe build).  usage: r4_big.sh [tag] [notests]
set -o pipefail
TAG=${1:-big}
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
if [ "$2" != "notests" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_timeout.py \
  tests/test_gpu_accuracy.py tests/test_shard.py -x -v --timeout 300 --timeout-method thread -k "big or wide or C5 or split or quarter or timeout or eight" \
  > gpurun_out/r4/${TAG}_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r4/${TAG}_tests.log | tail -40; [ $rc -eq 0 ] || { grep -E "^E " gpurun_out/r4/${TAG}_tests.log | head -30; exit $rc; }
fi
timeout -k 10 300 python -u tools/c5_pieces.py 2>&1 | tee gpurun_out/r4/${TAG}_pieces.txt || exit 1
GPK_LIB_PATH=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib/libgpk_trace.so timeout -k 10 300 python -u tools/big_timeline.py 2>&1 | tee gpurun_out/r4/${TAG}_timeline.txt
