#!/bin/bash
# round 4: new tests first (timeout path, chain in 2-rank groups), then the whole GPU suite,
# then the CPU-baseline calibration at the reference's own configs (profiles/r4_cpu_calibration.json)
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_timeout.py "tests/test_shard.py::test_group_chain_path_two_ranks" \
  -x -v --timeout 120 --timeout-method thread > gpurun_out/r4/new_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r4/new_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4/gpu_suite.log 2>&1
rc=$?; tail -5 gpurun_out/r4/gpu_suite.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r4/gpu_suite.log | head -30; exit $rc; }
if [ "$1" = "calib" ]; then
  timeout -k 10 400 python -u tools/cpu_calibration.py --seconds 10 --out gpurun_out/r4/cpu_calibration.json > gpurun_out/r4/calib.log 2>&1
  rc=$?; tail -3 gpurun_out/r4/calib.log; exit $rc
fi
