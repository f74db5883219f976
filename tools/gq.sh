set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_fastgraph.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/q6_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/q6_pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/q6_pytest.log | head -30; exit 1; fi
