# round 5: the C5 128-wide update on the pipelined tile loop and the uint8 variant gather -- the
# class / quarter-tile / wide tests, then the C5 kernel-parameter split with exact contractions
# (the A/B against the previous tree's library was run by an earlier version of this script:
# profiles/r5_c5_inv_ab.txt)
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dclass.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "quarter or wide or dclass or class or big or C5" -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r5/inv_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r5/inv_tests.log | tail -40
[ $rc -eq 0 ] || { grep -E "^E " gpurun_out/r5/inv_tests.log | head -30; exit 1; }
export OMP_NUM_THREADS=16
timeout -k 10 900 python -u tools/c5_kp_split.py C5 --axis 2
