#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_accuracy.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -q -m gpu -x --timeout 300 --timeout-method thread -k "C5 or c5 or big or large or 1600 or 2048" > gpurun_out/r3g_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r3g_pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/r3g_pytest.log | head -30; exit 1; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3g_bench.json 2> gpurun_out/r3g_bench.err || { tail -20 gpurun_out/r3g_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3g_bench.json')); print(d['value'], json.dumps(d['large_factors']))"
