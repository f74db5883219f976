set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kron3.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/q4_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/q4_pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/q4_pytest.log | head -30; exit 1; fi
