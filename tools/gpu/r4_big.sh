#!/bin/bash
# round 4: the large-factor inverse (blocked-Cholesky pivot + forward-substitution panel):
# big-path tests, C5 accuracy vs the yardstick, then the pieces' timings
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_timeout.py \
  tests/test_gpu_accuracy.py tests/test_shard.py -x -v --timeout 300 --timeout-method thread -k "big or wide or C5 or split or quarter or timeout or eight" \
  > gpurun_out/r4/big_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r4/big_tests.log | tail -40; [ $rc -eq 0 ] || { grep -E "^E " gpurun_out/r4/big_tests.log | head -30; exit $rc; }
timeout -k 10 300 python -u tools/c5_pieces.py 2>&1 | tee gpurun_out/r4/c5_pieces.txt
