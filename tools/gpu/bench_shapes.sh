# step-path tests, then the bench at the driver's shape (20 steps, 5 warm-up) and the default
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fastgraph.py tests/test_gpu_golden.py tests/test_abi.py tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_shapes.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_shapes.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error|Timeout" gpurun_out/pytest_shapes.log | head -30; exit 1; fi
for a in "--steps 20 --warmup 5" "--steps 20 --warmup 5" "--steps 500 --warmup 20"; do
  timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-large > gpurun_out/bs.json 2>/dev/null || { echo bench failed; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bs.json')); print('$a', round(d['value'],1), round(d['ms_per_step'],4), d['step1_per_call']['value'])"
done
