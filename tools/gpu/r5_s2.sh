# round 5: fast-graph / accuracy / fullsize GPU tests, then the C4 bench with the train_regime field
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_fastgraph.py tests/test_gpu_accuracy.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r5/s2_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r5/s2_tests.log | tail -40
[ $rc -eq 0 ] || { grep -E "^E " gpurun_out/r5/s2_tests.log | head -30; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 200 --no-large --no-cpu-baseline > gpurun_out/r5/bench_w200.json 2> gpurun_out/r5/bench_w200.err || { tail -20 gpurun_out/r5/bench_w200.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r5/bench_w200.json').read().splitlines()[-1]);print('W=200', {k:d[k] for k in ('value','ms_per_step','train_regime','step_graph')})"
