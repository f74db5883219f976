set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_shard.py tests/test_gpu_fullsize.py -x -v --timeout 150 --timeout-method thread -m gpu 2>&1 | tee gpurun_out/r5/shard_tests.log | grep -E "PASSED|FAILED|ERROR|Timeout|^E " 
