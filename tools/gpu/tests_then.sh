# all GPU tests, then the script named by $1 (if the tests did not abort)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/pytest_gpu.log | head -30; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest aborted rc=$rc"; exit 1; fi
[ -n "$1" ] && bash "$@"
