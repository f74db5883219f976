# chain iteration: chain tests, C2 + C4 timelines (probe build), C2 stage times, a short C4 bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_chain_multi.py tests/test_gpu_fastgraph.py tests/test_gpu_dclass.py tests/test_gpu_golden.py tests/test_gpu_dropin.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_chain.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_chain.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error|Timeout" gpurun_out/pytest_chain.log | head -30; exit 1; fi
timeout -k 10 120 python tools/timeline.py --config C2 --steps 3 > gpurun_out/tl_c2.txt 2>&1 &&
timeout -k 10 120 python tools/timeline.py --config C4 --steps 5 > gpurun_out/tl_c4.txt 2>&1 &&
timeout -k 10 120 python tools/run_steps.py --config C2 --steps 50 > gpurun_out/c2_stages.txt 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-large --steps 500 > gpurun_out/quick_bench.json 2> gpurun_out/quick_bench.err || { echo step failed; tail -5 gpurun_out/*.err gpurun_out/tl_*.txt; exit 1; }
head -1 gpurun_out/c2_stages.txt
python3 -c "import json; d=json.load(open('gpurun_out/quick_bench.json')); print('C4', d['value'], d['kernels_us'], d['step1_per_call'])"
